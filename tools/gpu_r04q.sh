#!/bin/bash
# K3 at <= 96 VGPRs for every instantiation (UPK_K3_WPE=5) vs one directional
# sample only (default): configs[2] regions pass and configs[4] replicates
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04q}; mkdir -p "$F"; cd "$R" || exit 1
for r in 1 2; do
  for w in hg19-nondir1 hg19mm9-32rep; do
    st=30; [ $w = hg19mm9-32rep ] && st=8
    for v in base k3all5; do
      L=""; [ $v != base ] && L=$R/exp/libunipeak_hip_$v.so
      UNIPEAK_LIB=$L timeout -k 10 300 python bench.py --workload $w --steps $st --warmup 2 --no-cpu-baseline > "$F/b_${w}_${v}_$r.json" 2> "$F/b_${w}_${v}_$r.err" || { tail -5 "$F/b_${w}_${v}_$r.err"; exit 1; }
      python -c "import json; d=json.loads(open('$F/b_${w}_${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$w $v', d['value'], d['ms_per_step'], d.get('regions'), 'iso', r.get('isolated_ms'))"
    done
  done
done
echo r04q-ok
