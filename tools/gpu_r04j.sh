#!/bin/bash
# configs[1] kernel timeline: what the GPU runs between consecutive K1a's
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04j}; mkdir -p "$F"; cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$F/trace" -o run -- python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline > "$F/bench.json" 2> "$F/bench.err" || { tail -5 "$F/bench.err"; exit 1; }
python3 tools/timeline_stats.py "$F/trace" 30 > "$F/timeline_stats.json" && cat "$F/timeline_stats.json"
python3 tools/timeline.py "$F/trace" 60 > "$F/timeline.txt"
echo r04j-ok
