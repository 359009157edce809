#!/bin/bash
# A/B of (library variant, environment) pairs in one call, so every variant
# runs on the same box: ab.sh "base|UNIPEAK_X=1" "pf|" ...  (variant "base" =
# the in-tree library, otherwise unipeak_amd/lib/libunipeak_hip_<v>.so from
# tools/build_variant.sh).  Bench N=1 (+ a simulated 8-GPU rank unless
# NO_SIM=1); REPS alternating rounds (default 1).  WORKLOAD selects the workload.
R="${GRAFT_REPO_ROOT:?}"; mkdir -p "$R/gpurun_out/ab"
WL="--workload ${WORKLOAD:-hg19-dir1}"
for rep in $(seq 1 "${REPS:-1}"); do
i=0
for spec in "$@"; do
  i=$((i+1))
  v=${spec%%|*}; e=${spec#*|}
  lib=$R/unipeak_amd/lib/libunipeak_hip_$v.so; [ "$v" = base ] && lib=$R/unipeak_amd/lib/libunipeak_hip.so
  o=$R/gpurun_out/ab/r${rep}_$i
  env $e UNIPEAK_LIB=$lib timeout -k 10 200 python "$R/bench.py" $WL --no-cpu-baseline --steps 30 --warmup 3 > "$o.json" 2> "$o.err" || { tail -3 "$o.err"; exit 1; }
  if [ -z "$NO_SIM" ]; then
    env $e UNIPEAK_LIB=$lib UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=4 timeout -k 10 200 python "$R/bench.py" $WL --no-cpu-baseline --steps 40 --warmup 3 > "${o}_n8.json" 2>/dev/null || exit 1
  fi
  echo "[$spec] $(python -c "
import json, os
d=json.loads(open('$o.json').read().strip().splitlines()[-1]); r=d['roofline']
s=''
if os.path.exists('${o}_n8.json'):
    e=json.load(open('${o}_n8.json')); s='| n8r4 %.4f k1a %.4f' % (e['ms_per_step'], e['k1a_ms'])
print(d['value'], d['ms_per_step'], 'k1a', r['kernel_ms'], 'iso', r['isolated_ms'], s)")"
done
done
