#!/bin/bash
# A/B of environment settings: ab_envs.sh "A=1 B=2" "A=0" ...  (bench N=1 +
# one simulated 8-GPU rank each; WORKLOAD selects the bench workload)
R="${GRAFT_REPO_ROOT:?}"; mkdir -p "$R/gpurun_out"
WL="--workload ${WORKLOAD:-hg19-dir1}"
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 200 python "$R/bench.py" $WL --no-cpu-baseline --steps 30 --warmup 3 > "$R/gpurun_out/abe_$i.json" 2> "$R/gpurun_out/abe_$i.err" || { tail -3 "$R/gpurun_out/abe_$i.err"; exit 1; }
  env $v UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=4 timeout -k 10 200 python "$R/bench.py" $WL --no-cpu-baseline --steps 40 --warmup 3 > "$R/gpurun_out/abe8_$i.json" 2>/dev/null || exit 1
  echo "[$v] $(python -c "
import json
d=json.loads(open('$R/gpurun_out/abe_$i.json').read().strip().splitlines()[-1]); r=d['roofline']
e=json.load(open('$R/gpurun_out/abe8_$i.json'))
print(d['value'], d['ms_per_step'], 'k1a', r['kernel_ms'], 'iso', r['isolated_ms'], '| n8r4', e['ms_per_step'], e['k1a_ms'], e['phases_ms'])")"
done
