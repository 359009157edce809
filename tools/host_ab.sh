#!/bin/bash
# Host cost per pass on one rank of the 8-GPU plan: launch sub-phases of
# bench.py under variants (env assignments in $VARIANTS, ';'-separated).
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"
F=$R/gpurun_out/host_ab
mkdir -p "$F"
cd "$R" || exit 1
IFS=';' read -ra VS <<< "${VARIANTS:-X=0}"
for rep in 1 2; do
for v in "${VS[@]}"; do
  n=$(echo "$v" | tr ' =' '__')
  env $v UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=${RANK8:-4} timeout -k 10 120 python bench.py --steps ${STEPS:-200} --warmup 5 --no-cpu-baseline > "$F/${n}_$rep.json" 2> "$F/${n}_$rep.err" || exit 1
  echo "$v: $(grep -o '"ms_per_step": [0-9.]*' "$F/${n}_$rep.json") $(grep -h 'per-step phases' "$F/${n}_$rep.err")"
done
done
