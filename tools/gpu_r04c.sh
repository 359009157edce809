#!/bin/bash
# round 4: copy-kernel probe, then the escape-bound K1a on the pooled workloads
# and configs[1] (A/B against round 3's K1a times)
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04c}; mkdir -p "$F"; cd "$R" || exit 1
true
true
timeout -k 10 600 python -u -m pytest tests/test_gpu_tracks.py tests/test_gpu_genome.py -k "tracks or escape or configs3 or configs4_hg19mm9_32_samples" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$F/pytest.log" 2>&1 || { grep -E "FAILED|Error|assert" "$F/pytest.log" | head -20; tail -5 "$F/pytest.log"; exit 1; }
tail -1 "$F/pytest.log"
for w in hg19-dir1 hg19-8s1c hg19mm9-32rep hg19mm9-32s; do
  st=10; [ $w = hg19-dir1 ] || st=5
  timeout -k 10 400 python bench.py --workload $w --steps $st --warmup 1 --no-cpu-baseline > "$F/bench_$w.json" 2> "$F/bench_$w.err" || { tail -5 "$F/bench_$w.err"; exit 1; }
  python -c "
import json; d=json.load(open('$F/bench_$w.json')); r=d['roofline']
print('$w', d['value'], d['ms_per_step'], d['regions'], r['isolated_ms'])"
done
echo gpu-ok
