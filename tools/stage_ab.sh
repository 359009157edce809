#!/bin/bash
# A/B of K3 record delivery: staged + DMA copy (UNIPEAK_STAGE=1, v=0) vs K3 writing host memory (default, v=1)
R=$GRAFT_REPO_ROOT
cd $R
for k in 1 2; do
for v in 0 1; do
  UNIPEAK_STAGE=$((1-v)) timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/st1_$v.json 2>/dev/null || exit 1
  UNIPEAK_STAGE=$((1-v)) UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=4 timeout -k 10 120 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/st8_$v.json 2>/dev/null || exit 1
  echo "no_stage=$v n1 $(python tools/jsum.py gpurun_out/st1_$v.json) | n8r4 $(python -c "import json;d=json.load(open('gpurun_out/st8_$v.json'));print(d['ms_per_step'], d['warmup_timings_ms'])")"
done; done
