#!/bin/bash
# launch-shape knobs on the final build, configs[1], same box, two rounds
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04s}; mkdir -p "$F"; cd "$R" || exit 1
for r in 1 2; do
  for v in default k1a2 chains4 chains2; do
    E="UNIPEAK_NONE=1"
    case $v in k1a2) E="UNIPEAK_K1A_PER_CU=2";; chains4) E="UNIPEAK_CHAINS=4";; chains2) E="UNIPEAK_CHAINS=2";; esac
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > "$F/b_${v}_$r.json" 2> "$F/b_${v}_$r.err" || { tail -5 "$F/b_${v}_$r.err"; exit 1; }
    python -c "import json; d=json.loads(open('$F/b_${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], 'k1a', r.get('kernel_ms'))"
  done
done
echo r04s-ok
