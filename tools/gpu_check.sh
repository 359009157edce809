#!/bin/bash
# Full GPU check: every -m gpu test, smoke, default bench line, configs[2]
# pipeline bench, and rocprofv3 kernel stats of the default bench.  Results
# under gpurun_out/<tag>/; the first failing step ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"
TAG=${1:-check}
F=$R/gpurun_out/$TAG
mkdir -p "$F"
cd "$R" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$F/pytest.log" 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|assert" "$F/pytest.log" | head -20; tail -5 "$F/pytest.log"; exit 1; }
tail -1 "$F/pytest.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$F/smoke.log" 2>&1 || { cat "$F/smoke.log"; exit 1; }
cat "$F/smoke.log"
timeout -k 10 300 python bench.py > "$F/bench.json" 2> "$F/bench.err" || { tail -5 "$F/bench.err"; exit 1; }
cut -c1-600 "$F/bench.json"
timeout -k 10 300 python bench.py --workload hg19-shift --steps 10 --warmup 2 --no-cpu-baseline > "$F/bench_shift.json" 2> "$F/bench_shift.err" || { tail -5 "$F/bench_shift.err"; exit 1; }
cut -c1-400 "$F/bench_shift.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace" -o p -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$F/trace.log" 2>&1 || { tail "$F/trace.log"; exit 1; }
echo check-ok
