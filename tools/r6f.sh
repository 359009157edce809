#!/bin/bash
# tests touching K1a (cold fields kernel), K3 many samples, then the bench
set -o pipefail
T=${1:-r6f}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_index.py tests/test_gpu_plane.py tests/test_gpu_unit.py tests/test_gpu_tracks.py tests/test_gpu_keys.py tests/test_gpu_q11_heads.py > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline > gpurun_out/$T/bench_$rep.json 2> gpurun_out/$T/bench_$rep.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['ms_per_step'], d['value'], r['kernel_ms'], r['isolated_ms'], d['warm']['ms_per_step'], d['single_pass_ms']['no_index']['median'])" gpurun_out/$T/bench_$rep.json
done
cd /tmp && export TMPDIR=/tmp
UNIPEAK_BENCH_LEGS=cold timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/$T/sq" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/$T/sq.log" 2>&1 || exit 1
python3 "$GRAFT_REPO_ROOT/tools/sq_kernels.py" "$GRAFT_REPO_ROOT/gpurun_out/$T/sq" > "$GRAFT_REPO_ROOT/gpurun_out/$T/sq_counters.json"
echo done
