#!/bin/bash
# K3L peak window per dword: parity (forced on, heavy path forced too), cuts, A/B
set -o pipefail
T=${1:-r6q}
R=$GRAFT_REPO_ROOT
mkdir -p gpurun_out/$T
UNIPEAK_K3_LANE=2 timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_keys.py tests/test_gpu_unit.py tests/test_gpu_k3.py tests/test_quirks.py tests/test_gpu_genome.py tests/test_gpu_tracks.py > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
UNIPEAK_K3_LANE=2 UNIPEAK_K3L_HEAVY=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_unit.py tests/test_gpu_k3.py > gpurun_out/$T/pytest_heavy.log 2>&1 || { tail -40 gpurun_out/$T/pytest_heavy.log; exit 1; }
tail -1 gpurun_out/$T/pytest_heavy.log
for cut in 4 5 0; do
  UNIPEAK_K3_LANE=2 UNIPEAK_K3L_CUT=$cut UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 timeout -k 10 200 python $R/bench.py --steps 10 --no-cpu-baseline > gpurun_out/$T/cut_$cut.json 2> gpurun_out/$T/cut_$cut.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cut', sys.argv[2], d['roofline']['isolated_ms']['k3'])" gpurun_out/$T/cut_$cut.json $cut
done
E="UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0"
REPS=2 tools/ab.sh "base|$E" "base|$E UNIPEAK_K3_LANE=0" | sed "s/UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0//"
