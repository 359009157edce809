#!/bin/bash
# round 4: the 8-rank rehearsal (every rank on device 0, rank 0's merged
# records vs N=1 byte for byte) for configs[1] and configs[3], and one PMC
# FETCH_SIZE / WRITE_SIZE pair on a configs[1] 8-GPU-plan rank shard
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/${1:-r04f}; mkdir -p "$F"; cd "$R" || exit 1
NS="8" WS="hg19-dir1 hg19-8s1c" timeout -k 10 900 tools/rehearse.sh > "$F/rehearse.jsonl" 2> "$F/rehearse.err" || { tail -20 "$F/rehearse.err"; cat "$F/rehearse.jsonl"; exit 1; }
cat "$F/rehearse.jsonl"
cp gpurun_out/rehearse/*.json "$F/" 2>/dev/null
cd /tmp && export TMPDIR=/tmp
UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=0 timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$F/sim_fetch" -o p -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$F/sim_fetch.log" 2>&1 || { tail "$F/sim_fetch.log"; exit 1; }
UNIPEAK_SIM_WORLD=8 UNIPEAK_SIM_RANK=0 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$F/sim_write" -o p -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$F/sim_write.log" 2>&1 || { tail "$F/sim_write.log"; exit 1; }
tail -1 "$F/sim_fetch.log"
echo gpu-ok
