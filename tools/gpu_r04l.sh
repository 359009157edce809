#!/bin/bash
# upper bounds: configs[1] step with K1b's blocks free / K3 free (wrong
# regions; experiment only), beside the real library, same box
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04l}; mkdir -p "$F"; cd "$R" || exit 1
for r in 1 2; do
  for v in real nok1b nok3; do
    L=""; [ $v != real ] && L=$R/exp/libunipeak_hip_$v.so
    UNIPEAK_LIB=$L timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > "$F/b_${v}_$r.json" 2> "$F/b_${v}_$r.err" || { tail -5 "$F/b_${v}_$r.err"; exit 1; }
    python -c "import json; d=json.loads(open('$F/b_${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], 'k1a', r.get('kernel_ms'), 'iso', r.get('isolated_ms'))"
  done
done
echo r04l-ok
