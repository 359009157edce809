#!/bin/bash
# round 4: K1q (threshold <= 0 in parallel) parity + timing, the escape-track
# mask A/B, and the default bench
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04e}; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_replay.py tests/test_cli.py tests/test_multidev.py tests/test_gpu_tracks.py "tests/test_gpu_genome.py::test_configs0_chr21_cli_threshold_zero" "tests/test_gpu_genome.py::test_configs3_hg19_pooled_with_control_units" -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider -rA > "$F/pytest.log" 2>&1 || { grep -E "FAILED|Error|assert" "$F/pytest.log" | head -30; tail -5 "$F/pytest.log"; exit 1; }
tail -1 "$F/pytest.log"
timeout -k 10 600 python tools/q11_probe.py chr21 0 > "$F/q11_chr21.json" 2> "$F/q11_chr21.err" || { tail -5 "$F/q11_chr21.err"; cat "$F/q11_chr21.json"; exit 1; }
cat "$F/q11_chr21.json"
for w in hg19-dir1 hg19-8s1c hg19mm9-32s; do
  st=10; [ $w = hg19-dir1 ] || st=5
  timeout -k 10 400 python bench.py --workload $w --steps $st --warmup 1 --no-cpu-baseline > "$F/bench_$w.json" 2> "$F/bench_$w.err" || { tail -5 "$F/bench_$w.err"; exit 1; }
  python -c "
import json; d=json.load(open('$F/bench_$w.json')); r=d['roofline']
print('$w', d['value'], d['ms_per_step'], d['regions'], r['isolated_ms'], 'copy', r['hbm_copy_GBps'])"
done
echo gpu-ok
