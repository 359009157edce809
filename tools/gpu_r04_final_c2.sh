#!/bin/bash
# round-4 final set, part C2: the 8-rank rehearsal (records vs N=1) alone
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-final_c2}; mkdir -p "$F"; cd "$R" || exit 1
NS="8" WS="hg19-dir1 hg19-8s1c hg19mm9-32rep" timeout -k 10 1000 tools/rehearse.sh > "$F/rehearse.jsonl" 2> "$F/rehearse.err" || { tail -20 "$F/rehearse.err"; cat "$F/rehearse.jsonl"; exit 1; }
cat "$F/rehearse.jsonl"
echo final-c2-ok
