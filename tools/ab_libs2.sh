#!/bin/bash
# A/B of variant builds: bench (N=1) + isolated breakdown + one simulated
# 8-GPU rank.  usage: [WORKLOAD=hg19-nondir1] ab_libs2.sh base NAME...
R="${GRAFT_REPO_ROOT:?}"; mkdir -p "$R/gpurun_out"
WL="--workload ${WORKLOAD:-hg19-dir1}"
for v in "$@"; do
  lib=$R/unipeak_amd/lib/libunipeak_hip_$v.so; [ "$v" = base ] && lib=$R/unipeak_amd/lib/libunipeak_hip.so
  UNIPEAK_LIB=$lib timeout -k 10 200 python "$R/bench.py" $WL --no-cpu-baseline --steps 30 --warmup 3 > "$R/gpurun_out/ab_$v.json" 2> "$R/gpurun_out/ab_$v.err" || { tail -3 "$R/gpurun_out/ab_$v.err"; exit 1; }
  UNIPEAK_LIB=$lib UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=4 timeout -k 10 200 python "$R/bench.py" $WL --no-cpu-baseline --steps 40 --warmup 3 > "$R/gpurun_out/ab8_$v.json" 2>/dev/null || exit 1
  echo "$v $(python -c "
import json
d=json.loads(open('$R/gpurun_out/ab_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
e=json.load(open('$R/gpurun_out/ab8_$v.json'))
print(d['value'], d['ms_per_step'], 'k1a', r['kernel_ms'], 'iso', r['isolated_ms'], '| n8r4', e['ms_per_step'], e['warmup_timings_ms'])")"
done
