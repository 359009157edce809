#!/bin/bash
# One GPU session: gpu tests, smoke, bench (N=1), simulated ranks of N=8.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
NS="${SIM_NS:-8}" tools/sim_ranks.sh > gpurun_out/sim.log 2>&1 || { echo sim failed; tail gpurun_out/sim.log; exit 1; }
cat gpurun_out/sim.log
