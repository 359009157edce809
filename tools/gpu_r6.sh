#!/bin/bash
# Round-6 measurement set (results under gpurun_out/<tag>/): the bench's
# cold + warm legs with GPU_MAX_HW_QUEUES 4 and 8 alternating (two pairs),
# rocprofv3 kernel-trace stats of the default bench, K1a (cold: the 2-bit
# fields stream, kModeScreenF = mode 3) PMC traffic, and SQ counters of the
# cold leg's kernels.  Usage: tools/gpu_r6.sh TAG [skip-ab]
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"
TAG=${1:-r6}
F=$R/gpurun_out/$TAG
mkdir -p "$F"
cd "$R" || exit 1
if [ "$2" != "skip-ab" ]; then
  for rep in 1 2; do
    for q in 4 8; do
      UNIPEAK_HWQ=$q timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline > "$F/ab_q${q}_$rep.json" 2> "$F/ab_q${q}_$rep.err" || exit 1
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['value'], d['warm']['ms_per_step'], d['value_warm'])" "$F/ab_q${q}_$rep.json" "q$q#$rep"
    done
  done
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace" -o p -- python3 "$R/bench.py" --steps 50 --no-cpu-baseline > "$F/trace.json" 2> "$F/trace.err" || exit 1
UNIPEAK_BENCH_LEGS=cold timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$F/fetch" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/fetch.log" 2>&1 || exit 1
UNIPEAK_BENCH_LEGS=cold timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$F/write" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/write.log" 2>&1 || exit 1
python3 "$R/tools/pmc_traffic.py" "$F/fetch" "$F/write" "scan_kernel<1, 0, false, false, 3>" 1547846991 "$F/k1a_pmc_traffic.json" || exit 1
UNIPEAK_BENCH_LEGS=cold timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d "$F/sq" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/sq.log" 2>&1 || exit 1
python3 "$R/tools/sq_kernels.py" "$F/sq" > "$F/sq_counters.json" || exit 1
echo r6-ok
