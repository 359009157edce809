#!/bin/bash
# round-4 final set, part C: the 8-GPU plans' rank shards run alone (compute
# side of the scaling runs), and the 8-rank rehearsal (records vs N=1)
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-final_c3}; mkdir -p "$F"; cd "$R" || exit 1


for w in hg19-dir1 hg19-8s1c hg19mm9-32rep; do
  st=200; [ $w = hg19-dir1 ] || st=20
  for r in 0 1 2 3 4 5 6 7; do
    UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=$r timeout -k 10 300 python bench.py --workload $w --steps $st --warmup 3 --no-cpu-baseline > "$F/sim8_${w}_r$r.json" 2> /dev/null || exit 1
  done
  python -c "
import json
v=[json.load(open('$F/sim8_${w}_r%d.json' % r))['ms_per_step'] for r in range(8)]
print('$w sim8', [round(x, 4) for x in v], 'max', max(v))"
done
NS="8" WS="hg19-dir1 hg19-8s1c hg19mm9-32rep" timeout -k 10 900 tools/rehearse.sh > "$F/rehearse.jsonl" 2> "$F/rehearse.err" || { tail -20 "$F/rehearse.err"; cat "$F/rehearse.jsonl"; exit 1; }
cat "$F/rehearse.jsonl"
echo final-c-ok
