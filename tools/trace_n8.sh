#!/bin/bash
# Kernel timeline of one simulated rank of the 8-GPU plan (env passes through)
R="${GRAFT_REPO_ROOT:?}"
OUT=$R/gpurun_out/trace_${1:-x}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=4 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/n8" -o t -- python3 "$R/bench.py" --steps 12 --warmup 2 --no-cpu-baseline > "$OUT/n8.log" 2>&1 || exit 1
python3 "$R/tools/timeline.py" "$OUT/n8" 200 > "$OUT/timeline_n8.txt"
