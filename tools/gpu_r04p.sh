#!/bin/bash
# the default bench line (50 steps, CPU baselines) and the rocprofv3 stats of
# the same command
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04p}; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 400 python bench.py > "$F/bench_full.json" 2> "$F/bench_full.err" || { tail -5 "$F/bench_full.err"; exit 1; }
python -c "import json; d=json.loads(open('$F/bench_full.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], d['steps'], r['frac'], r['kernel_ms'], r['traffic'], r['traffic_source'], r['isolated_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace" -o p -- python3 "$R/bench.py" --no-cpu-baseline > "$F/trace.log" 2>&1 || { tail "$F/trace.log"; exit 1; }
cp "$(ls "$F"/trace/*kernel_stats.csv "$F"/trace/*/*kernel_stats.csv 2>/dev/null | head -1)" "$F/bench_kernel_stats.csv"
head -4 "$F/bench_kernel_stats.csv" | cut -c1-140
echo r04p-ok
