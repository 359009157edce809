#!/bin/bash
# K1b per-wave phase clocks of a debug build (tools/build_variant.sh dbgt
# -DUPK_DEBUG_TIMES): N=1 bench and one simulated rank of the 8-GPU plan
R="${GRAFT_REPO_ROOT:?}"; mkdir -p "$R/gpurun_out"
export UNIPEAK_DEBUG_COUNTS=1 UNIPEAK_LIB=$R/unipeak_amd/lib/libunipeak_hip_${1:-dbgt}.so
timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --steps 2 --warmup 1 > "$R/gpurun_out/dbgt.json" 2> "$R/gpurun_out/dbgt.err" || exit 1
grep "K1b clocks" "$R/gpurun_out/dbgt.err" | tail -1
UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=4 timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --steps 2 --warmup 1 > "$R/gpurun_out/dbgt8.json" 2> "$R/gpurun_out/dbgt8.err" || exit 1
grep "K1b clocks" "$R/gpurun_out/dbgt8.err" | tail -1
