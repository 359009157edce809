#!/bin/bash
# slow-mode hypothesis: chain kernels serialised on shared hardware queues
R=$GRAFT_REPO_ROOT; F=$R/gpurun_out/r6s; mkdir -p $F
run() { tag=$1; shift; env "$@" UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 timeout -k 10 300 python $R/bench.py --no-cpu-baseline --steps 30 > $F/$tag.json 2> $F/$tag.err || { tail -3 $F/$tag.err; exit 1; }
  echo "$tag $(grep 'cold:' $F/$tag.err)"; }
for rep in 1 2; do
run default$rep X=1
run chains1_$rep UNIPEAK_CHAINS=1
run hwq2_$rep UNIPEAK_HWQ=2
run hwq16_$rep UNIPEAK_HWQ=16
done
