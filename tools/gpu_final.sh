#!/bin/bash
# Round profile set (results under gpurun_out/<tag>/): every GPU test, smoke,
# the default bench line (CPU baselines), the other BASELINE workloads,
# rocprofv3 kernel stats of the bench, K1a PMC traffic (FETCH_SIZE and
# WRITE_SIZE passes), SQ counter passes, and the 8-GPU plans' rank shards.
# Steps chained: the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; TAG=${1:-final}; F=$R/gpurun_out/$TAG; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$F/pytest.log" 2>&1 || { grep -E "FAILED|Error" "$F/pytest.log" | head; tail -3 "$F/pytest.log"; exit 1; }
tail -1 "$F/pytest.log"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$F/smoke.log" 2>&1 || { cat "$F/smoke.log"; exit 1; }
cat "$F/smoke.log"
timeout -k 10 300 python bench.py > "$F/bench.json" 2> "$F/bench.err" || { tail -5 "$F/bench.err"; exit 1; }
cut -c1-300 "$F/bench.json"
for w in hg19-nondir1 hg19-8s1c hg19-shift; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > "$F/bench_$w.json" 2> "$F/bench_$w.err" || { tail -3 "$F/bench_$w.err"; exit 1; }
  cut -c1-160 "$F/bench_$w.json"
done
timeout -k 10 300 python bench.py --bw 150 --steps 10 --warmup 2 --no-cpu-baseline > "$F/bench_bw150.json" 2> "$F/bench_bw150.err" || { tail -3 "$F/bench_bw150.err"; exit 1; }
cut -c1-160 "$F/bench_bw150.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace" -o p -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$F/trace.log" 2>&1 || { tail "$F/trace.log"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$F/fetch" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/fetch.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$F/write" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/write.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$F/pmc_a" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/pmc_a.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR --output-format csv -d "$F/pmc_b" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/pmc_b.log" 2>&1 || exit 1
cd "$R" || exit 1
for w in hg19-dir1 hg19-8s1c hg19mm9-32s; do
  st=200; [ $w = hg19-dir1 ] || st=30
  for r in 0 1 2 3 4 5 6 7; do
    UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=$r timeout -k 10 300 python bench.py --workload $w --steps $st --warmup 3 --no-cpu-baseline > "$F/sim8_${w}_r$r.json" 2> /dev/null || exit 1
  done
  python -c "
import json
v=[json.load(open('$F/sim8_${w}_r%d.json' % r))['ms_per_step'] for r in range(8)]
print('$w sim8', [round(x, 4) for x in v], 'max', max(v))"
done
timeout -k 10 600 python bench.py --workload hg19mm9-32s --steps 5 --warmup 1 --no-cpu-baseline > "$F/bench_hg19mm9-32s.json" 2> "$F/bench_32s.err" || exit 1
cut -c1-160 "$F/bench_hg19mm9-32s.json"
echo final-ok
