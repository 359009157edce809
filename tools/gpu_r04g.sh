#!/bin/bash
# round 4: A/B of K1a's escape detection (tile index, scalar vs bytes, VALU)
# on configs[1] and configs[3], two alternating rounds; K1a isolated times
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04g}; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_tracks.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > "$F/pytest.log" 2>&1 || { grep -E "FAILED|Error|assert" "$F/pytest.log" | head -20; exit 1; }
tail -1 "$F/pytest.log"
for rep in 1 2; do
 for v in base escvalu; do
  lib=$R/unipeak_amd/lib/libunipeak_hip_$v.so; [ $v = base ] && lib=$R/unipeak_amd/lib/libunipeak_hip.so
  for w in hg19-dir1 hg19-8s1c; do
    st=20; [ $w = hg19-dir1 ] || st=6
    UNIPEAK_LIB=$lib timeout -k 10 300 python bench.py --workload $w --steps $st --warmup 2 --no-cpu-baseline > "$F/${v}_${w}_$rep.json" 2> /dev/null || exit 1
    python -c "
import json; d=json.load(open('$F/${v}_${w}_$rep.json')); r=d['roofline']
print('$rep $v $w', d['value'], d['ms_per_step'], r['isolated_ms']['k1a'], r['isolated_ms']['k1b_k1x'])"
  done
 done
done
echo gpu-ok
