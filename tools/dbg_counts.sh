#!/bin/bash
# K1 work counters of a debug build (tools/build_variant.sh dbg -DUPK_DEBUG_COUNTS)
R="${GRAFT_REPO_ROOT:?}"; mkdir -p "$R/gpurun_out"
UNIPEAK_DEBUG_COUNTS=1 UNIPEAK_LIB=$R/unipeak_amd/lib/libunipeak_hip_dbg.so timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --steps 2 --warmup 1 > "$R/gpurun_out/dbg.json" 2> "$R/gpurun_out/dbg.err" || exit 1
grep "unipeak_hip: K1" "$R/gpurun_out/dbg.err" | tail -2
