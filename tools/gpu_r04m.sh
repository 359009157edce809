#!/bin/bash
# occupancy beside K1a: K3 at 96 VGPRs (two K3 waves fit beside three K1a
# waves per SIMD), K1b at 96, K1a at two workgroups per CU; configs[1], same box
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04m}; mkdir -p "$F"; cd "$R" || exit 1
for r in 1 2; do
  for v in real k3w5 k1bw5 k1a2; do
    L=""; E=""
    case $v in k3w5|k1bw5) L=$R/exp/libunipeak_hip_$v.so;; k1a2) E="UNIPEAK_K1A_PER_CU=2";; esac
    env $E UNIPEAK_LIB=$L timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > "$F/b_${v}_$r.json" 2> "$F/b_${v}_$r.err" || { tail -5 "$F/b_${v}_$r.err"; exit 1; }
    python -c "import json; d=json.loads(open('$F/b_${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], 'k1a', r.get('kernel_ms'), 'iso', r.get('isolated_ms'))"
  done
done
echo r04m-ok
