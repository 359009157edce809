#!/bin/bash
# configs[1] 8-GPU plan rank shards with K1a at two workgroups per CU vs three
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04t}; mkdir -p "$F"; cd "$R" || exit 1
for v in 3 2; do
  for r in 0 1 2 3 4 5 6 7; do
    UNIPEAK_K1A_PER_CU=$v UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=$r timeout -k 10 120 python bench.py --steps 200 --warmup 3 --no-cpu-baseline > "$F/sim8_k1a${v}_r$r.json" 2> /dev/null || exit 1
  done
  python -c "
import json
v=[json.load(open('$F/sim8_k1a${v}_r%d.json' % r))['ms_per_step'] for r in range(8)]
print('k1a_per_cu $v', [round(x, 4) for x in v], 'max', max(v))"
done
echo r04t-ok
