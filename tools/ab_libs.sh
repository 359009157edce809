#!/bin/bash
# A/B of variant builds (UNIPEAK_LIB) on the bench and on rank 0 of an 8-GPU plan
R=$GRAFT_REPO_ROOT
for v in "$@"; do
  lib=$R/unipeak_amd/lib/libunipeak_hip$v.so
  UNIPEAK_LIB=$lib timeout -k 10 200 python $R/bench.py --no-cpu-baseline > $R/gpurun_out/ab$v.json 2> $R/gpurun_out/ab$v.err || exit 1
  UNIPEAK_LIB=$lib UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=0 timeout -k 10 200 python $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/ab8$v.json 2>/dev/null || exit 1
  echo "variant '$v': $(python $R/tools/jsum.py $R/gpurun_out/ab$v.json) | n8 r0: $(python -c "import json;d=json.load(open('$R/gpurun_out/ab8$v.json'));print(d['ms_per_step'], d['warmup_timings_ms'])")"
done
