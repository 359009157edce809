#!/bin/bash
# kernel-trace timeline of the cold leg alone (no single passes after it)
set -o pipefail
T=${1:-r6g}
F=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $F
cd /tmp && export TMPDIR=/tmp
UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace" -o p -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 50 --no-cpu-baseline > "$F/trace.json" 2> "$F/trace.err" || exit 1
python3 "$GRAFT_REPO_ROOT/tools/timeline_stats.py" "$F/trace" 30 3 > "$F/timeline.json" || exit 1
cat "$F/timeline.json" | head -60
