#!/bin/bash
# final build: configs[2] lines (nondirectional K3 change), cold + warm; the strand_shift pipeline
set -o pipefail
R=$GRAFT_REPO_ROOT; F=$R/gpurun_out/r6zz; mkdir -p $F; cd $R || exit 1
for w in hg19-nondir1 hg19-shift; do
  st=20; [ $w = hg19-shift ] && st=10
  timeout -k 10 400 python bench.py --workload $w --steps $st --warmup 2 --no-cpu-baseline > $F/bench_$w.json 2> $F/bench_$w.err || { tail -3 $F/bench_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], (d.get('warm') or {}).get('value'), (d.get('warm') or {}).get('ms_per_step'), d['roofline'].get('isolated_ms'))" $F/bench_$w.json $w
done
