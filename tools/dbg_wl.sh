#!/bin/bash
# K1b phase clocks (variant dbgt, -DUPK_DEBUG_TIMES) and exact-block counts
# (variant dbgc, -DUPK_DEBUG_COUNTS) of one bench workload: dbg_wl.sh WORKLOAD
R="${GRAFT_REPO_ROOT:?}"; mkdir -p "$R/gpurun_out/dbg"
for v in dbgt dbgc; do
  UNIPEAK_DEBUG_COUNTS=1 UNIPEAK_LIB=$R/unipeak_amd/lib/libunipeak_hip_$v.so timeout -k 10 200 python "$R/bench.py" --workload "$1" --no-cpu-baseline --steps 2 --warmup 1 > "$R/gpurun_out/dbg/$1_$v.json" 2> "$R/gpurun_out/dbg/$1_$v.err" || exit 1
  grep "unipeak_hip: K1" "$R/gpurun_out/dbg/$1_$v.err" | tail -3
done
