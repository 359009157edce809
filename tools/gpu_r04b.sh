#!/bin/bash
# round 4: the tests not reached by r04a's run (gzip, multi-device), then the
# bench lines for configs[1], [3] and [4] (both generators)
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04b}; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gzip.py tests/test_multidev.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rA > "$F/pytest.log" 2>&1 || { grep -E "FAILED|Error|assert" "$F/pytest.log" | head -20; tail -5 "$F/pytest.log"; exit 1; }
tail -1 "$F/pytest.log"
timeout -k 10 300 python bench.py --no-cpu-baseline > "$F/bench.json" 2> "$F/bench.err" || { tail -5 "$F/bench.err"; exit 1; }
cut -c1-300 "$F/bench.json"
for w in hg19-8s1c hg19mm9-32rep hg19mm9-32s; do
  timeout -k 10 400 python bench.py --workload $w --steps 5 --warmup 1 --no-cpu-baseline > "$F/bench_$w.json" 2> "$F/bench_$w.err" || { tail -5 "$F/bench_$w.err"; exit 1; }
  python -c "
import json; d=json.load(open('$F/bench_$w.json')); r=d['roofline']
print('$w', d['value'], d['ms_per_step'], d['regions'], r['isolated_ms'], 'copy', r['hbm_copy_GBps'])"
done
echo gpu-ok
