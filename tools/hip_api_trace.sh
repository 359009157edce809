#!/bin/bash
# HIP API durations of a bench run (host cost per pass): rocprofv3
# --hip-trace --stats of N=1 and of one rank of the 8-GPU plan.
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"
F=$R/gpurun_out/hiptrace
mkdir -p "$F"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d "$F/n1" -o p -- python3 "$R/bench.py" --steps 100 --warmup 3 --no-cpu-baseline > "$F/n1.log" 2>&1 || exit 1
UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=4 timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d "$F/n8r4" -o p -- python3 "$R/bench.py" --steps 100 --warmup 3 --no-cpu-baseline > "$F/n8r4.log" 2>&1 || exit 1
echo trace-ok
