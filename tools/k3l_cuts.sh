#!/bin/bash
# K3L phase cuts: isolated K3 time of the bench's blocking passes per cut (records wrong by design)
R=$GRAFT_REPO_ROOT
for cut in 0 1 2 3 4 5; do
  UNIPEAK_K3_LANE=2 UNIPEAK_K3L_CUT=$cut UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 timeout -k 10 200 python $R/bench.py --steps 10 --no-cpu-baseline > $R/gpurun_out/k3cut_$cut.json 2> $R/gpurun_out/k3cut_$cut.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cut', sys.argv[2], d['roofline']['isolated_ms'])" $R/gpurun_out/k3cut_$cut.json $cut
done
cd /tmp && export TMPDIR=/tmp
UNIPEAK_K3_LANE=2 UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS --output-format csv -d "$R/gpurun_out/k3sq" -o p -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$R/gpurun_out/k3sq.log" 2>&1 || exit 1
python3 "$R/tools/sq_kernels.py" "$R/gpurun_out/k3sq" | python3 -c "import json,sys; d=json.load(sys.stdin); print({k: v for k, v in d.items() if 'stats1L' in k or k.startswith('K3')})"
