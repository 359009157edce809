#!/bin/bash
# closing check on the final build: every GPU test, smoke, the default bench line, its kernel stats
set -o pipefail
R=$GRAFT_REPO_ROOT; F=$R/gpurun_out/${1:-r6z}; mkdir -p $F; cd $R || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $F/pytest.log 2>&1 || { grep -E "FAILED|Error" $F/pytest.log | head; tail -3 $F/pytest.log; exit 1; }
tail -1 $F/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { cat $F/smoke.log; exit 1; }
cat $F/smoke.log
timeout -k 10 400 python bench.py > $F/bench.json 2> $F/bench.err || { tail -5 $F/bench.err; exit 1; }
grep -h "cold:\|warm:" $F/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace" -o p -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$F/trace.log" 2>&1 || { tail "$F/trace.log"; exit 1; }
grep -h "cold:\|warm:" $F/trace.log
