#!/bin/bash
# Round-3 batch: targeted GPU tests (TESTS), the default bench line, K1a PMC
# traffic (FETCH_SIZE and WRITE_SIZE passes) and SQ counter passes over the
# bench; results under gpurun_out/<tag>/, the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"
TAG=${1:-r03b}
F=$R/gpurun_out/$TAG
mkdir -p "$F"
cd "$R" || exit 1
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$F/pytest.log" 2>&1 || { grep -E "FAILED|Error" "$F/pytest.log" | head -20; tail -3 "$F/pytest.log"; exit 1; }
  tail -1 "$F/pytest.log"
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS} > "$F/bench.json" 2> "$F/bench.err" || { tail -5 "$F/bench.err"; exit 1; }
cut -c1-300 "$F/bench.json"
[ -n "$NO_PMC" ] && { echo batch-ok; exit 0; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace" -o p -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$F/trace.log" 2>&1 || { tail "$F/trace.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$F/fetch" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/fetch.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$F/write" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/write.log" 2>&1 || exit 1
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$F/pmc_$name" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/pmc_$name.log" 2>&1
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
run b SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR || exit 1
echo batch-ok
