#!/bin/bash
# A/B of variant builds (tools/build_variant.sh NAME ...): K1 probe + bench
# line + one simulated 8-GPU rank per variant.  usage: ab_k1.sh base NAME...
R="${GRAFT_REPO_ROOT:?}"; mkdir -p "$R/gpurun_out"
for v in "$@"; do
  lib=$R/unipeak_amd/lib/libunipeak_hip_$v.so; [ "$v" = base ] && lib=$R/unipeak_amd/lib/libunipeak_hip.so
  UNIPEAK_LIB=$lib timeout -k 10 200 python "$R/tools/k1_probe.py" --reps 7 --modes synthetic,zeros > "$R/gpurun_out/k1p_$v.json" 2> "$R/gpurun_out/k1p_$v.err" || { tail -3 "$R/gpurun_out/k1p_$v.err"; exit 1; }
  UNIPEAK_LIB=$lib timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --steps 20 --warmup 3 > "$R/gpurun_out/ab_$v.json" 2> "$R/gpurun_out/ab_$v.err" || { tail -3 "$R/gpurun_out/ab_$v.err"; exit 1; }
  UNIPEAK_LIB=$lib UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=4 timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --steps 30 --warmup 3 > "$R/gpurun_out/ab8_$v.json" 2>/dev/null || exit 1
  echo "$v probe $(cat "$R/gpurun_out/k1p_$v.json")"
  echo "$v bench $(python "$R/tools/jsum.py" "$R/gpurun_out/ab_$v.json") | n8r4 $(python -c "import json;d=json.load(open('$R/gpurun_out/ab8_$v.json'));print(d['ms_per_step'], d['warmup_timings_ms'])")"
done
