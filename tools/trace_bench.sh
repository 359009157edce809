#!/bin/bash
# Kernel timeline of the N=1 bench (rocprofv3 kernel trace, csv) and of one
# simulated rank of the 8-GPU plan; summarised by tools/timeline.py.
R="${GRAFT_REPO_ROOT:?}"
OUT=$R/gpurun_out/trace_${1:-x}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/n1" -o t -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/n1.log" 2>&1 || exit 1
UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=4 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/n8" -o t -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/n8.log" 2>&1 || exit 1
python3 "$R/tools/timeline.py" "$OUT/n1" > "$OUT/timeline_n1.txt"; python3 "$R/tools/timeline.py" "$OUT/n8" > "$OUT/timeline_n8.txt"
tail -40 "$OUT/timeline_n1.txt"; tail -25 "$OUT/timeline_n8.txt"
