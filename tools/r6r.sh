#!/bin/bash
# the default bench line vs the A/B settings (cold leg slow in the default run?)
set -o pipefail
R=$GRAFT_REPO_ROOT; F=$R/gpurun_out/r6r; mkdir -p $F
run() { tag=$1; shift; env "$@" timeout -k 10 300 python $R/bench.py $BARGS > $F/$tag.json 2> $F/$tag.err || { tail -3 $F/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d.get('warm',{}).get('ms_per_step'), d['roofline']['kernel_ms'])" $F/$tag.json $tag; grep "cold:" $F/$tag.err; }
BARGS="--no-cpu-baseline" run default X=1
BARGS="--no-cpu-baseline" run cold_only UNIPEAK_BENCH_LEGS=cold
BARGS="--no-cpu-baseline --steps 30" run steps30 X=1
BARGS="--no-cpu-baseline --steps 30 --warmup 3" run ab_like UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0
BARGS="--no-cpu-baseline" run default2 X=1
