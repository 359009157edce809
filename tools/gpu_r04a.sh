#!/bin/bash
# round 4, first GPU call: the new replicate-mode tests, the full configs[4]
# parity test, then the default bench line and the configs[4] replicate bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"; F=$R/gpurun_out/r04a; mkdir -p "$F"; cd "$R" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_unit.py -k "replicate or synthetic" tests/test_gpu_genome.py -k "replicate or synthetic or in_oracle or configs4" -x -v --timeout 400 --timeout-method thread -p no:cacheprovider > "$F/pytest.log" 2>&1 || { grep -E "FAILED|Error|assert" "$F/pytest.log" | head -20; tail -5 "$F/pytest.log"; exit 1; }
grep -E "PASSED|identical" "$F/pytest.log" | tail -12
timeout -k 10 300 python bench.py --no-cpu-baseline > "$F/bench.json" 2> "$F/bench.err" || { tail -5 "$F/bench.err"; exit 1; }
cut -c1-400 "$F/bench.json"
timeout -k 10 400 python bench.py --workload hg19mm9-32rep --steps 5 --warmup 1 --no-cpu-baseline > "$F/bench_32rep.json" 2> "$F/bench_32rep.err" || { tail -5 "$F/bench_32rep.err"; exit 1; }
cut -c1-1200 "$F/bench_32rep.json"
echo r04a-ok
