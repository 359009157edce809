#!/bin/bash
R="${GRAFT_REPO_ROOT:?}"; mkdir -p "$R/gpurun_out"
for pc in 2 3; do
for v in base a6 a8 b5 a8b5; do
  lib=$R/unipeak_amd/lib/libunipeak_hip_$v.so; [ "$v" = base ] && lib=$R/unipeak_amd/lib/libunipeak_hip.so
  UNIPEAK_K1A_PER_CU=$pc UNIPEAK_LIB=$lib timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --steps 30 --warmup 3 > "$R/gpurun_out/abv_$v.json" 2> "$R/gpurun_out/abv_$v.err" || { tail -3 "$R/gpurun_out/abv_$v.err"; exit 1; }
  UNIPEAK_K1A_PER_CU=$pc UNIPEAK_LIB=$lib UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=4 timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --steps 40 --warmup 3 > "$R/gpurun_out/abv8_$v.json" 2>/dev/null || exit 1
  echo "pc=$pc $v bench $(python "$R/tools/jsum.py" "$R/gpurun_out/abv_$v.json") | n8r4 $(python -c "import json;d=json.load(open('$R/gpurun_out/abv8_$v.json'));print(d['ms_per_step'], d['k1a_ms'], d['warmup_timings_ms'])")"
done
done
