#!/bin/bash
# PMC passes over a short bench run (one counter group per pass) plus the
# kernel-trace summary; outputs under gpurun_out/pmc_<tag>/
R=$GRAFT_REPO_ROOT
TAG=${1:-x}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $R/gpurun_out/pmc_$TAG/$name -o p -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_$TAG/$name.log 2>&1
}
mkdir -p $R/gpurun_out/pmc_$TAG
run a SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES || exit $?
run b SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD || exit $?
run c SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_SMEM GRBM_GUI_ACTIVE || exit $?
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pmc_$TAG/trace -o p -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/pmc_$TAG/trace.log 2>&1 || exit $?
