#!/bin/bash
# round-4 final set, part A: every GPU test, smoke, the default bench line
# (CPU baselines included) and the other BASELINE workloads at N=1
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-final_a}; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > "$F/pytest_gpu.log" 2>&1 || { grep -E "FAILED|Error|assert" "$F/pytest_gpu.log" | head -20; tail -3 "$F/pytest_gpu.log"; exit 1; }
tail -1 "$F/pytest_gpu.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$F/smoke.log" 2>&1 || { cat "$F/smoke.log"; exit 1; }
cat "$F/smoke.log"
timeout -k 10 400 python bench.py > "$F/bench_full.json" 2> "$F/bench_full.err" || { tail -5 "$F/bench_full.err"; exit 1; }
cut -c1-250 "$F/bench_full.json"
for w in hg19-nondir1 hg19-8s1c hg19-shift hg19mm9-32rep hg19mm9-32s; do
  st=10; case $w in hg19mm9*) st=5;; esac
  timeout -k 10 400 python bench.py --workload $w --steps $st --warmup 2 --no-cpu-baseline > "$F/bench_$w.json" 2> "$F/bench_$w.err" || { tail -3 "$F/bench_$w.err"; exit 1; }
  python -c "
import json; d=json.load(open('$F/bench_$w.json')); r=d['roofline']
print('$w', d['value'], d['ms_per_step'], d.get('regions'), r.get('isolated_ms'))"
done
timeout -k 10 300 python bench.py --bw 150 --steps 10 --warmup 2 --no-cpu-baseline > "$F/bench_bw150.json" 2> "$F/bench_bw150.err" || exit 1
timeout -k 10 300 python bench.py --bw 300 --steps 10 --warmup 2 --no-cpu-baseline > "$F/bench_bw300.json" 2> "$F/bench_bw300.err" || exit 1
python -c "
import json
for b in ('150', '300'):
    d=json.load(open('$F/bench_bw'+b+'.json')); print('bw', b, d['value'], d['ms_per_step'], d['roofline']['isolated_ms'])"
echo final-a-ok
