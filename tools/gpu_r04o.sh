#!/bin/bash
# K1b: dead words skip the key and the LDS store (new) vs every word
# (UPK_K1B_ALL_WORDS); new + K3 at 96 VGPRs.  Tests first, then a same-box A/B
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04o}; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$F/pytest.log" 2>&1 || { tail -30 "$F/pytest.log"; exit 1; }
tail -1 "$F/pytest.log"
for r in 1 2 3; do
  for v in new allwords k3w5; do
    L=""; [ $v != new ] && L=$R/exp/libunipeak_hip_$v.so
    UNIPEAK_LIB=$L timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > "$F/b_${v}_$r.json" 2> "$F/b_${v}_$r.err" || { tail -5 "$F/b_${v}_$r.err"; exit 1; }
    python -c "import json; d=json.loads(open('$F/b_${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], 'k1a', r.get('kernel_ms'), 'iso', r.get('isolated_ms'))"
  done
done
echo r04o-ok
