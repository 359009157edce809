#!/bin/bash
# Kernel timeline (rocprofv3 kernel trace, csv) of one simulated rank of an
# N-GPU plan (bench.py UNIPEAK_SIM_WORLD) -- per-kernel durations and the
# gaps between them inside a step.
N=${1:-8}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/trace_n$N
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
UNIPEAK_SIM_WORLD=$N UNIPEAK_SIM_RANK=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT -o t -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/log 2>&1
