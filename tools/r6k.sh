#!/bin/bash
# K3L parity (forced on for every test: UNIPEAK_K3_LANE=2) + A/B at N=1 and a simulated 8-GPU rank
set -o pipefail
T=${1:-r6k}
mkdir -p gpurun_out/$T
UNIPEAK_K3_LANE=2 timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_keys.py tests/test_gpu_unit.py tests/test_quirks.py tests/test_gpu_index.py tests/test_gpu_plane.py tests/test_gpu_tracks.py tests/test_gpu_genome.py tests/test_cli.py > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
E="UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0"
REPS=2 tools/ab.sh "base|$E UNIPEAK_K3_LANE=2" "base|$E UNIPEAK_K3_LANE=0" | sed 's/UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0//'
