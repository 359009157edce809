#!/bin/bash
# Every BASELINE workload at N=1 plus simulated rank shards of the 8-GPU
# plans (UNIPEAK_SIM_WORLD=8, the slowest-planned rank), one JSON each under
# gpurun_out/<tag>/; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"
TAG=${1:-wl}
F=$R/gpurun_out/$TAG
mkdir -p "$F"
cd "$R" || exit 1
for w in hg19-nondir1 hg19-8s1c hg19-shift; do
  timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline > "$F/bench_$w.json" 2> "$F/bench_$w.err" || { tail -5 "$F/bench_$w.err"; exit 1; }
  python -c "import json;d=json.load(open('$F/bench_$w.json'));print('$w', d['value'], d['ms_per_step'], d['roofline'].get('isolated_ms'))"
done
for w in hg19-dir1 hg19-8s1c hg19mm9-32s; do
  for r in ${SIM_RANKS:-0 1 2 3 4 5 6 7}; do
    UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=$r timeout -k 10 300 python bench.py --workload $w --steps ${SIM_STEPS:-50} --warmup 3 --no-cpu-baseline > "$F/sim8_${w}_r$r.json" 2> "$F/sim8_${w}_r$r.err" || { tail -5 "$F/sim8_${w}_r$r.err"; exit 1; }
  done
  python -c "
import json
v=[json.load(open('$F/sim8_${w}_r%d.json' % r))['ms_per_step'] for r in [int(x) for x in '${SIM_RANKS:-0 1 2 3 4 5 6 7}'.split()]]
print('$w sim8 ranks ms', v, 'max', max(v))"
done
echo workloads-ok
