#!/bin/bash
# K1a one-track: exact sums + bitmap-gated escape bits (new) vs the 2 x
# popcount first stage (UPK_K1A_BOUND2); tests first, then a same-box A/B
# and K1a's VALU count
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04n}; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_tracks.py tests/test_gpu_unit.py tests/test_gpu_keys.py tests/test_gpu_genome.py -m gpu -x -q --timeout 300 --timeout-method thread > "$F/pytest.log" 2>&1 || { tail -30 "$F/pytest.log"; exit 1; }
tail -1 "$F/pytest.log"
for r in 1 2; do
  for v in new bound2; do
    L=""; [ $v = bound2 ] && L=$R/exp/libunipeak_hip_bound2.so
    UNIPEAK_LIB=$L timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > "$F/b_${v}_$r.json" 2> "$F/b_${v}_$r.err" || { tail -5 "$F/b_${v}_$r.err"; exit 1; }
    python -c "import json; d=json.loads(open('$F/b_${v}_$r.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], 'k1a', r.get('kernel_ms'), 'iso', r.get('isolated_ms'))"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d "$F/pmc" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/pmc.log" 2>&1 || exit 1
python3 "$R/tools/sq_summary.py" "$F/sq.json" "new K1a" "$F/pmc" || exit 1
echo r04n-ok
