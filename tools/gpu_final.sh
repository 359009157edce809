#!/bin/bash
# Round profile set, in stages (one gpurun call each; results under
# gpurun_out/<tag>/; the first failure ends the stage):
#   tools/gpu_final.sh TAG tests   every GPU test, smoke, the default bench line
#                                  (CPU baselines), the other BASELINE workloads
#   tools/gpu_final.sh TAG bench   the bench lines and probes alone
#   tools/gpu_final.sh TAG prof    rocprofv3 kernel stats of the default bench,
#                                  K1a PMC traffic (FETCH_SIZE / WRITE_SIZE passes,
#                                  gfx950-corrected), SQ counter passes
#   tools/gpu_final.sh TAG sim     the 8-GPU plans' rank shards (one GPU), and
#                                  the 8-rank rehearsal through the bare launcher
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; TAG=${1:-final}; STAGE=${2:-tests}; F=$R/gpurun_out/$TAG; mkdir -p "$F"; cd "$R" || exit 1
line() { python -c "
import json, sys
d = json.loads(open('$1').read().strip().splitlines()[-1]); r = d['roofline']
print('$2', d['value'], 'Gbp/s', d['ms_per_step'], 'ms/step; K1a', r['kernel_ms'], 'frac', r['frac'], 'iso', r.get('isolated_ms'))"; }
case $STAGE in
tests)
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$F/pytest.log" 2>&1 || { grep -E "FAILED|Error" "$F/pytest.log" | head; tail -3 "$F/pytest.log"; exit 1; }
  tail -1 "$F/pytest.log"
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$F/smoke.log" 2>&1 || { cat "$F/smoke.log"; exit 1; }
  cat "$F/smoke.log"
  ;&
bench)
  timeout -k 10 400 python bench.py > "$F/bench.json" 2> "$F/bench.err" || { tail -5 "$F/bench.err"; exit 1; }
  line "$F/bench.json" hg19-dir1
  for w in hg19-nondir1 hg19-8s1c hg19-shift hg19mm9-32rep hg19mm9-32s; do
    st=20; case $w in hg19-shift) st=10;; esac
    timeout -k 10 400 python bench.py --workload $w --steps $st --warmup 2 --no-cpu-baseline > "$F/bench_$w.json" 2> "$F/bench_$w.err" || { tail -3 "$F/bench_$w.err"; exit 1; }
    line "$F/bench_$w.json" $w
  done
  for b in 150 300; do
    timeout -k 10 300 python bench.py --bw $b --steps 20 --warmup 2 --no-cpu-baseline > "$F/bench_bw$b.json" 2> "$F/bench_bw$b.err" || { tail -3 "$F/bench_bw$b.err"; exit 1; }
    line "$F/bench_bw$b.json" bw$b
  done
  # the paths outside K1: wide kernels, the replay, -r 0 with heads
  timeout -k 10 300 python tools/replay_probe.py chr21 > "$F/replay_probe_chr21.jsonl" 2> "$F/replay_probe.err" || exit 1
  timeout -k 10 300 python tools/q11_heads_probe.py > "$F/q11_heads_probe.json" 2> "$F/q11_heads_probe.err" || exit 1
  cat "$F/q11_heads_probe.json"
  ;;
prof)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace" -o p -- python3 "$R/bench.py" --steps 20 --warmup 3 --no-cpu-baseline > "$F/trace.log" 2>&1 || { tail "$F/trace.log"; exit 1; }
  UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$F/fetch" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/fetch.log" 2>&1 || exit 1
  UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$F/write" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/write.log" 2>&1 || exit 1
  python3 "$R/tools/pmc_traffic.py" "$F/fetch" "$F/write" k1a_fields_kernel 1547846991 "$F/k1a_pmc_traffic.json" || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d "$F/pmc_a" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/pmc_a.log" 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR --output-format csv -d "$F/pmc_b" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/pmc_b.log" 2>&1 || exit 1
  echo prof-ok
  ;;
sim)
  for w in hg19-dir1 hg19-8s1c hg19mm9-32rep; do
    st=200; [ $w = hg19-dir1 ] || st=30; [ $w = hg19mm9-32rep ] && st=10
    for r in 0 1 2 3 4 5 6 7; do
      UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=$r timeout -k 10 300 python bench.py --workload $w --steps $st --warmup 3 --no-cpu-baseline > "$F/sim8_${w}_r$r.json" 2> /dev/null || exit 1
    done
    python -c "
import json
d=[json.load(open('$F/sim8_${w}_r%d.json' % r)) for r in range(8)]
v=[x['ms_per_step'] for x in d]
wv=[x.get('legs_ms_per_step', {}).get('warm', float('nan')) for x in d]
print('$w sim8 cold', [round(x, 4) for x in v], 'max', max(v), '| warm max', max(wv))"
  done
  NS=8 WS="hg19-dir1 hg19-8s1c" bash tools/rehearse.sh > "$F/rehearse.jsonl" 2>&1 || { tail -5 "$F/rehearse.jsonl"; exit 1; }
  cat "$F/rehearse.jsonl"
  ;;
esac
echo "$STAGE-ok"
