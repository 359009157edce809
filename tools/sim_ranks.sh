#!/bin/bash
# Compute side of N-GPU strong scaling on a one-GPU box: run every rank's
# shard of the N-rank LPT plan alone (bench.py, UNIPEAK_SIM_WORLD), one
# process per (N, rank).  The slowest rank bounds the N-GPU step.
OUT=${OUT:-gpurun_out/sim}
mkdir -p $OUT
WL=${WL:-hg19-dir1}
for N in ${NS:-2 4 8}; do
  for ((r = 0; r < N; r++)); do
    UNIPEAK_SIM_WORLD=$N UNIPEAK_SIM_RANK=$r timeout -k 10 120 python bench.py --workload $WL --steps ${STEPS:-20} --warmup 3 \
      --no-cpu-baseline > $OUT/${WL}_n${N}_r${r}.json 2> $OUT/${WL}_n${N}_r${r}.err || exit $?
    cat $OUT/${WL}_n${N}_r${r}.json
  done
done
