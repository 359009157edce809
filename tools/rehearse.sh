#!/bin/bash
# The N-rank bench path (`bench.py --gpus N` launches the ranks itself through
# torch.distributed.run, StepBoard, node-shared record slots, rank
# 0's merge in global unit order) end to end on a one-GPU box: every rank on
# device 0 (UNIPEAK_SHARE_GPU), gloo for the setup collectives (RCCL refuses
# two ranks on one GPU).  Rank 0's merged records and exptSums of the last
# step (UNIPEAK_BENCH_DUMP) must equal N=1's byte for byte.
# usage: NS="2 4 8" WS="hg19-dir1 hg19-8s1c" tools/rehearse.sh
R="${GRAFT_REPO_ROOT:?}"; cd "$R" || exit 1; D=gpurun_out/rehearse; mkdir -p $D
for W in ${WS:-hg19-dir1 hg19-8s1c}; do
  ST=20; [ "$W" = hg19-dir1 ] || ST=6
  UNIPEAK_BENCH_DUMP=$D/${W}_n1.npz timeout -k 10 300 python bench.py --workload $W --steps $ST --warmup 2 \
    --no-cpu-baseline > $D/${W}_n1.json 2> $D/${W}_n1.err || { tail -20 $D/${W}_n1.err; exit 1; }
  for N in ${NS:-2 4 8}; do
    UNIPEAK_BENCH_DUMP=$D/${W}_n$N.npz UNIPEAK_SHARE_GPU=1 UNIPEAK_DIST_BACKEND=gloo timeout -k 10 400 \
      python bench.py --workload $W --gpus $N --steps $ST --warmup 2 --no-cpu-baseline \
      > $D/${W}_n$N.json 2> $D/${W}_n$N.err || { tail -20 $D/${W}_n$N.err; exit 1; }
    python - "$D/${W}_n1.npz" "$D/${W}_n$N.npz" "$D/${W}_n$N.json" "$W" "$N" <<'EOF' || exit 1
import json, sys
import numpy as np
a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
same = a["recs"].tobytes() == b["recs"].tobytes() and a["counts"].tobytes() == b["counts"].tobytes()
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
print(json.dumps({"workload": sys.argv[4], "ranks": int(sys.argv[5]), "records": int(len(b["recs"])),
                  "records_and_exptsums_identical_to_n1": bool(same), "value": d["value"],
                  "ms_per_step": d["ms_per_step"], "note": "all ranks share one GPU: timing is not a scaling figure"}))
sys.exit(0 if same and len(b["recs"]) > 0 else 1)
EOF
  done
done
