#!/bin/bash
# what the GPU test suite leaves running before the bench (slow cold leg after it, 2 of 3 times)
set -o pipefail
R=$GRAFT_REPO_ROOT; F=$R/gpurun_out/r6y2; mkdir -p $F; cd $R || exit 1
ps -eo pid,ppid,pcpu,etime,cmd --sort=-pcpu | head -15 > $F/ps_before.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $F/pytest.log 2>&1 || { tail -3 $F/pytest.log; exit 1; }
tail -1 $F/pytest.log
ps -eo pid,ppid,pcpu,etime,cmd --sort=-pcpu | head -15 > $F/ps_after.txt
cat $F/ps_after.txt | cut -c1-150
ls /dev/shm | head > $F/shm_after.txt; cat $F/shm_after.txt
UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 > $F/b1.json 2> $F/b1.err || exit 1
grep 'cold:' $F/b1.err | cut -c1-100
ps -eo pid,ppid,pcpu,etime,cmd --sort=-pcpu | head -8 | cut -c1-150
UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 > $F/b2.json 2> $F/b2.err || exit 1
grep 'cold:' $F/b2.err | cut -c1-100
