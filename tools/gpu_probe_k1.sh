#!/bin/bash
# K1 probe on the GPU box: timings (synthetic vs zero tracks) and two PMC
# passes of instruction counters over the synthetic run.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline > $R/gpurun_out/bench.log 2>&1 || exit $?
timeout -k 10 300 python3 $R/tools/k1_probe.py > $R/gpurun_out/k1_probe.json 2> $R/gpurun_out/k1_probe.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/k1pmc_a -o p -- python3 $R/tools/k1_probe.py --reps 2 > $R/gpurun_out/k1pmc_a.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $R/gpurun_out/k1pmc_b -o p -- python3 $R/tools/k1_probe.py --reps 2 > $R/gpurun_out/k1pmc_b.log 2>&1 || exit $?
