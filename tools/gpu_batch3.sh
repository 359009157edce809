#!/bin/bash
# round-3 batch: every GPU test, then A/Bs (escape tiles, chain streams),
# the configs[2] pipeline and the replay probe; the first failure ends it
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/b3; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$F/pytest.log" 2>&1 || { grep -E "FAILED|Error" "$F/pytest.log" | head; tail -3 "$F/pytest.log"; exit 1; }
tail -1 "$F/pytest.log"
NO_SIM=1 WORKLOAD=hg19-8s1c tools/ab.sh "notile|" "base|" || exit 1
NO_SIM=1 REPS=2 tools/ab.sh "notile|" "base|" "bpf|" "base|UNIPEAK_CHAINS=3" "base|UNIPEAK_CHAINS=4" || exit 1
timeout -k 10 300 python bench.py --workload hg19-shift --steps 10 --warmup 2 --no-cpu-baseline > "$F/bench_shift.json" 2> "$F/bench_shift.err" || { tail -3 "$F/bench_shift.err"; exit 1; }
cut -c1-700 "$F/bench_shift.json"
timeout -k 10 300 python tools/replay_probe.py chr21 > "$F/replay.jsonl" 2> "$F/replay.err" || { tail -3 "$F/replay.err"; exit 1; }
cat "$F/replay.jsonl"
timeout -k 10 600 python bench.py --workload hg19mm9-32s --steps 5 --warmup 1 --no-cpu-baseline > "$F/bench_32s.json" 2> "$F/bench_32s.err" || { tail -3 "$F/bench_32s.err"; exit 1; }
cut -c1-400 "$F/bench_32s.json"
echo b3-ok
