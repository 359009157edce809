#!/bin/bash
# K3L heavy regions through the wave: region statistics, parity (forced on), A/B of the threshold
set -o pipefail
T=${1:-r6n}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
timeout -k 10 120 python tools/region_stats.py > gpurun_out/$T/region_stats.txt 2>&1 || { cat gpurun_out/$T/region_stats.txt; exit 1; }
cat gpurun_out/$T/region_stats.txt
UNIPEAK_K3_LANE=2 UNIPEAK_K3L_HEAVY=4 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_keys.py tests/test_gpu_unit.py tests/test_gpu_k3.py tests/test_quirks.py tests/test_gpu_genome.py > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
E="UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 UNIPEAK_K3_LANE=2"
REPS=2 tools/ab.sh "base|$E UNIPEAK_K3L_HEAVY=48" "base|$E UNIPEAK_K3L_HEAVY=24" "base|$E UNIPEAK_K3L_HEAVY=96" "base|$E UNIPEAK_K3L_HEAVY=100000" | sed 's/UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0//'
