#!/bin/bash
# K1a one-track popcount bound + escape bitmap: GPU tests, then a same-box
# A/B of configs[1] (new library vs UPK_NO_K1A_CHEAP), plus the timeline
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04k}; mkdir -p "$F"; cd "$R" || exit 1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$F/pytest.log" 2>&1 || { tail -30 "$F/pytest.log"; exit 1; }
tail -2 "$F/pytest.log"
for r in 1 2; do
  for v in new old; do
    L=""; [ $v = old ] && L=$R/exp/libunipeak_hip_nocheap.so
    UNIPEAK_LIB=$L timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > "$F/b_${v}_$r.json" 2> "$F/b_${v}_$r.err" || { tail -5 "$F/b_${v}_$r.err"; exit 1; }
    python -c "import json; d=json.loads(open('$F/b_${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], 'k1a', r.get('kernel_ms'), 'iso', r.get('isolated_ms'))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$F/trace" -o run -- python3 bench.py --steps 40 --warmup 3 --no-cpu-baseline > "$F/trace_bench.json" 2> "$F/trace_bench.err" || { tail -5 "$F/trace_bench.err"; exit 1; }
python3 tools/timeline_stats.py "$F/trace" 30 > "$F/timeline_stats.json" && cat "$F/timeline_stats.json"
echo r04k-ok
