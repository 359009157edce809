#!/bin/bash
# closing check of the final build: every GPU test, smoke, the default line,
# the workloads whose K3 changed, rocprofv3 stats of the default command
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04r}; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > "$F/pytest_gpu.log" 2>&1 || { grep -E "FAILED|Error|assert" "$F/pytest_gpu.log" | head -20; tail -3 "$F/pytest_gpu.log"; exit 1; }
tail -1 "$F/pytest_gpu.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$F/smoke.log" 2>&1 || { cat "$F/smoke.log"; exit 1; }
cat "$F/smoke.log"
timeout -k 10 400 python bench.py > "$F/bench_full.json" 2> "$F/bench_full.err" || { tail -5 "$F/bench_full.err"; exit 1; }
python -c "import json; d=json.loads(open('$F/bench_full.json').read().strip().splitlines()[-1]); r=d['roofline']; print('full', d['value'], d['ms_per_step'], d['steps'], r['frac'], r['kernel_ms'], r['isolated_ms'], d['cpu_baseline']['value'])"
for w in hg19-nondir1 hg19-shift hg19-8s1c hg19mm9-32rep; do
  st=10; case $w in hg19mm9*) st=5;; esac
  timeout -k 10 400 python bench.py --workload $w --steps $st --warmup 2 --no-cpu-baseline > "$F/bench_$w.json" 2> "$F/bench_$w.err" || { tail -3 "$F/bench_$w.err"; exit 1; }
  python -c "
import json; d=json.load(open('$F/bench_$w.json')); r=d.get('roofline') or {}
print('$w', d['value'], d['ms_per_step'], d.get('regions'), r.get('isolated_ms'))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace" -o p -- python3 "$R/bench.py" --no-cpu-baseline > "$F/trace.log" 2>&1 || { tail "$F/trace.log"; exit 1; }
cp "$(ls "$F"/trace/*kernel_stats.csv "$F"/trace/*/*kernel_stats.csv 2>/dev/null | head -1)" "$F/bench_kernel_stats.csv"
echo r04r-ok
