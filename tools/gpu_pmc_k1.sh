#!/bin/bash
# SQ counter passes and HBM traffic over a short bench run; per-kernel
# summary with tools/pmc_summary.py.  outputs under gpurun_out/pmcx_<tag>/
R="${GRAFT_REPO_ROOT:?}"
TAG=${1:-x}
mkdir -p "$R/gpurun_out/pmcx_$TAG"
cd /tmp && export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$R/gpurun_out/pmcx_$TAG/$name" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/pmcx_$TAG/$name.log" 2>&1
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit $?
run b SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR || exit $?
run c GRBM_GUI_ACTIVE GRBM_COUNT || exit $?
run f FETCH_SIZE || exit $?
run w WRITE_SIZE || exit $?
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmcx_$TAG" "scan_kernelILi1ELi0ELb0ELb0ELi2E" "scan_kernelILi1ELi0ELb0ELb0ELi1E" "stats_kernel" "seg_compact" > "$R/gpurun_out/pmcx_$TAG/summary.txt"
cat "$R/gpurun_out/pmcx_$TAG/summary.txt"
