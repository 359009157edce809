#!/bin/bash
# K3L parity (single-sample directional paths, ties, Q8, genome) + bench A/B vs stats1
set -o pipefail
T=${1:-r6h}
mkdir -p gpurun_out/$T
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_keys.py tests/test_gpu_unit.py tests/test_quirks.py tests/test_gpu_index.py tests/test_gpu_plane.py tests/test_gpu_tracks.py tests/test_gpu_genome.py > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
E="UNIPEAK_BENCH_SINGLE=0"
for rep in 1 2; do
  for k3 in 1 0; do
    env $E UNIPEAK_K3_LANE=$k3 timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline > gpurun_out/$T/b_${k3}_$rep.json 2> gpurun_out/$T/b_${k3}_$rep.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['ms_per_step'], d['value'], r['kernel_ms'], r['isolated_ms'], d['warm']['ms_per_step'], d['value_warm'], d['warm']['roofline']['isolated_ms'])" gpurun_out/$T/b_${k3}_$rep.json "k3lane=$k3"
  done
done
