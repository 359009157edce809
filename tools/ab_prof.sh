#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of variant
# builds on rank R of an N-GPU plan (bench.py UNIPEAK_SIM_WORLD; N=1: the
# whole bench workload).  usage: N=8 bash tools/ab_prof.sh "" _x
R=$GRAFT_REPO_ROOT
N=${N:-8}
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  OUT=$R/gpurun_out/abp$v
  rm -rf $OUT; mkdir -p $OUT
  UNIPEAK_LIB=$R/unipeak_amd/lib/libunipeak_hip$v.so UNIPEAK_SIM_WORLD=$N UNIPEAK_SIM_RANK=${RANK_SIM:-0} \
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o p -- python3 $R/bench.py --steps 30 --warmup 3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/log || exit 1
  echo "variant '$v' n$N: $(python3 $R/tools/kstats.py $(find $OUT -name 'p_kernel_stats.csv' | head -1)) | ms/step $(python3 -c "import json;print(json.load(open('$OUT/bench.json'))['ms_per_step'])")"
done
