#!/bin/bash
# Round-3 measurement batch (results under gpurun_out/<tag>/): new GPU tests,
# the default bench line (CPU baselines incl. all cores + end-to-end CLIs),
# the configs[2] full pipeline, rocprofv3 kernel stats of both, and SQ
# counter passes over the bench (K1a / K1b / K3).  Steps chained: the first
# failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"
TAG=${1:-r03c}
F=$R/gpurun_out/$TAG
mkdir -p "$F"
cd "$R" || exit 1
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$F/pytest.log" 2>&1 || { tail -20 "$F/pytest.log"; exit 1; }
  tail -1 "$F/pytest.log"
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > "$F/bench_full.json" 2> "$F/bench_full.err" || { tail -5 "$F/bench_full.err"; exit 1; }
cut -c1-400 "$F/bench_full.json"
timeout -k 10 300 python bench.py --workload hg19-shift --steps 10 --warmup 2 > "$F/bench_shift.json" 2> "$F/bench_shift.err" || { tail -5 "$F/bench_shift.err"; exit 1; }
cat "$F/bench_shift.json" | cut -c1-600
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace" -o p -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$F/trace.log" 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace_shift" -o p -- python3 "$R/bench.py" --workload hg19-shift --steps 5 --warmup 1 > "$F/trace_shift.log" 2>&1 || exit 1
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$F/pmc_$name" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/pmc_$name.log" 2>&1
}
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS || exit 1
run b SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR || exit 1
python3 "$R/tools/pmc_summary.py" "$F" "scan_kernelILi1ELi0ELb0ELb0ELi1E" "scan_kernelILi1ELi0ELb0ELb0ELi2E" "stats_kernel" "seg_compact" "xref" > "$F/pmc_summary.txt" || exit 1
echo batch-ok
