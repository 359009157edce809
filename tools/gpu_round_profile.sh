#!/bin/bash
# Round profile set (results under gpurun_out/final_<tag>/, copied into
# profiles/<tag>/ afterwards): pytest -m gpu, bench with CPU baseline, the
# other BASELINE workloads at N=1, the RCCL/shm bench path at world 1,
# simulated ranks of 2/4/8-GPU plans, rocprofv3 kernel-trace stats and the
# K1a PMC traffic of the bench.
set -o pipefail
R="${GRAFT_REPO_ROOT:?}"
TAG=${1:-r02}
F=$R/gpurun_out/final_$TAG
mkdir -p "$F"
cd "$R" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$F/pytest_gpu.log" 2>&1 || { tail -20 "$F/pytest_gpu.log"; exit 1; }
tail -1 "$F/pytest_gpu.log"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > "$F/bench_full.json" 2> "$F/bench_full.err" || exit 1
tail -1 "$F/bench_full.json" | cut -c1-300
for wl in hg19-nondir1 hg19-8s1c; do
  timeout -k 10 300 python bench.py --workload $wl --no-cpu-baseline > "$F/bench_$wl.json" 2> "$F/bench_$wl.err" || exit 1
done
UNIPEAK_BENCH_DIST=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 3 > "$F/bench_dist1.json" 2> "$F/bench_dist1.err" || exit 1
OUT=$F/sim NS="2 4 8" STEPS=200 tools/sim_ranks.sh > "$F/sim.log" 2>&1 || exit 1
python tools/sim_summary.py "$F/sim" "$F/bench_full.json" "$F/sim_ranks.json" || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$F/trace" -o p -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$F/trace.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$F/fetch" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/fetch.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$F/write" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$F/write.log" 2>&1 || exit 1
python3 "$R/tools/pmc_traffic.py" "$F/fetch" "$F/write" "scan_kernel<1, 0, false, false, 1>" 3095693983 "$F/k1a_pmc_traffic.json" || exit 1
timeout -k 10 300 rocprofv3 --hip-trace --stats --output-format csv -d "$F/hip" -o p -- python3 "$R/bench.py" --steps 100 --warmup 3 --no-cpu-baseline > "$F/hip.log" 2>&1 || exit 1
echo profile-ok
