#!/bin/bash
# round 4: NH <= 8 (bw <= 511 in the parallel scan) -- every GPU test, the
# replay probe (-b 300 / 511 / -r 0 timing), the escape-detection A/B
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04h}; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > "$F/pytest.log" 2>&1 || { grep -E "FAILED|Error|assert" "$F/pytest.log" | head -30; tail -5 "$F/pytest.log"; exit 1; }
tail -1 "$F/pytest.log"
timeout -k 10 300 python tools/replay_probe.py chr21 > "$F/replay_probe.jsonl" 2> "$F/replay_probe.err" || { tail -5 "$F/replay_probe.err"; exit 1; }
cat "$F/replay_probe.jsonl"
echo gpu-ok
