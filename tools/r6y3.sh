#!/bin/bash
# after the GPU suite: does the hardware-queue count change the slow (no-overlap) cold leg?
set -o pipefail
R=$GRAFT_REPO_ROOT; F=$R/gpurun_out/r6y3; mkdir -p $F; cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $F/pytest.log 2>&1 || { tail -3 $F/pytest.log; exit 1; }
tail -1 $F/pytest.log
for q in 8 4 16 2 8; do
  UNIPEAK_HWQ=$q UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > $F/q$q.json 2> $F/q$q.err || exit 1
  echo "hwq $q $(grep 'cold warmup' $F/q$q.err | cut -c15-70) | $(grep 'cold:' $F/q$q.err | cut -c1-60)"
done
