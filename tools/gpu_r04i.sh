#!/bin/bash
# round 4: K0 chain groups in parallel -- the replay / head-hit tests, then
# the configs[4] replicate bench (every unit takes the Q1 head replay)
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04i}; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_unit.py tests/test_gpu_replay.py tests/test_cli.py tests/test_multidev.py tests/test_gpu_pipeline.py "tests/test_gpu_genome.py::test_configs4_hg19mm9_32_replicates_full" "tests/test_gpu_genome.py::test_configs2_hg19_strand_shift_then_regions_cli" -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > "$F/pytest.log" 2>&1 || { grep -E "FAILED|Error|assert" "$F/pytest.log" | head -30; tail -5 "$F/pytest.log"; exit 1; }
tail -1 "$F/pytest.log"
for w in hg19mm9-32rep hg19-shift; do
  timeout -k 10 400 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > "$F/bench_$w.json" 2> "$F/bench_$w.err" || { tail -5 "$F/bench_$w.err"; exit 1; }
  python -c "
import json; d=json.load(open('$F/bench_$w.json')); r=d['roofline']
print('$w', d['value'], d['ms_per_step'], d.get('regions'), r.get('isolated_ms'), d.get('phases_ms'))"
done
echo gpu-ok
