#!/bin/bash
# GPU tests, two bench runs (value, ms/step, isolated breakdown, host phases)
# and the host A/B of one 8-GPU rank ($VARIANTS)
R="${GRAFT_REPO_ROOT:?}"; cd "$R" || exit 1; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_q.log 2>&1 || { tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -1 gpurun_out/pytest_q.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_q$i.json 2> gpurun_out/bench_q$i.err || { tail -20 gpurun_out/bench_q$i.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['isolated_ms'])" gpurun_out/bench_q$i.json
  grep phases gpurun_out/bench_q$i.err
done
[ -n "$VARIANTS" ] && bash tools/host_ab.sh
exit 0
