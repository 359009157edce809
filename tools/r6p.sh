#!/bin/bash
# K3L cuts: 2 staging, 6 + walk 1, 3 + walk 2, 7 full without the folded peak window, 0 full
R=$GRAFT_REPO_ROOT
for cut in 3 4 5 0; do
  UNIPEAK_K3_LANE=2 UNIPEAK_K3L_CUT=$cut UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 timeout -k 10 200 python $R/bench.py --steps 10 --no-cpu-baseline > $R/gpurun_out/k3cut_$cut.json 2> $R/gpurun_out/k3cut_$cut.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('cut', sys.argv[2], d['roofline']['isolated_ms']['k3'])" $R/gpurun_out/k3cut_$cut.json $cut
done
