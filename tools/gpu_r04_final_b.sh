#!/bin/bash
# round-4 final set, part B: rocprofv3 kernel stats of the default bench, the
# K1a PMC traffic (FETCH_SIZE and WRITE_SIZE passes), two SQ counter passes,
# and FETCH_SIZE / WRITE_SIZE on a configs[1] 8-GPU-plan rank shard
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-final_b}; mkdir -p "$F"; cd /tmp || exit 1; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace" -o p -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$F/trace.log" 2>&1 || { tail "$F/trace.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$F/fetch" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/fetch.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$F/write" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/write.log" 2>&1 || exit 1
python3 "$R/tools/pmc_traffic.py" "$F/fetch" "$F/write" "scan_kernel<1, 0, false, false, 1>" 1547846991 "$F/k1a_pmc_traffic.json" || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$F/pmc_a" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/pmc_a.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR --output-format csv -d "$F/pmc_b" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/pmc_b.log" 2>&1 || exit 1
UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$F/sim_fetch" -o p -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$F/sim_fetch.log" 2>&1 || exit 1
UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=0 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$F/sim_write" -o p -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$F/sim_write.log" 2>&1 || exit 1
tail -1 "$F/sim_fetch.log" | cut -c1-200
python3 "$R/tools/sq_summary.py" "$F/sq_counters.json" "rocprofv3 --pmc SQ counters per launch (mean over the bench passes; two passes of 8 counters), hg19 configs[1]" "$F/pmc_a" "$F/pmc_b" || exit 1
cp "$F"/trace/*kernel_stats.csv "$F/bench_kernel_stats.csv" 2>/dev/null || cp "$(ls "$F"/trace/*/*kernel_stats.csv | head -1)" "$F/bench_kernel_stats.csv"
echo final-b-ok
