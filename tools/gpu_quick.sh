#!/bin/bash
# Quick GPU check: bench (N=1, no CPU baseline), one simulated 8-GPU rank,
# then pytest -m gpu.  BENCH_ARGS / SKIP_TESTS override.
set -o pipefail
cd "${GRAFT_REPO_ROOT:?}"
mkdir -p gpurun_out
timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline --steps 20 --warmup 3} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=4 timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/sim8r4.json 2> gpurun_out/sim8r4.err || { echo sim failed; tail gpurun_out/sim8r4.err; exit 1; }
cat gpurun_out/sim8r4.json
[ -n "$SKIP_TESTS" ] && exit 0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
