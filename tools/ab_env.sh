#!/bin/bash
# A/B of an environment variable on the bench (N=1) and one simulated 8-GPU
# rank: ab_env.sh VAR v1 v2 ...
R="${GRAFT_REPO_ROOT:?}"; mkdir -p "$R/gpurun_out"
var=$1; shift
for v in "$@"; do
  env "$var=$v" timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --steps 30 --warmup 3 > "$R/gpurun_out/env_$v.json" 2> "$R/gpurun_out/env_$v.err" || { tail -3 "$R/gpurun_out/env_$v.err"; exit 1; }
  env "$var=$v" UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=4 timeout -k 10 200 python "$R/bench.py" --no-cpu-baseline --steps 40 --warmup 3 > "$R/gpurun_out/env8_$v.json" 2>/dev/null || exit 1
  echo "$var=$v bench $(python "$R/tools/jsum.py" "$R/gpurun_out/env_$v.json") | n8r4 $(python -c "import json;d=json.load(open('$R/gpurun_out/env8_$v.json'));print(d['ms_per_step'], d['k1a_ms'], d['warmup_timings_ms'])")"
done
