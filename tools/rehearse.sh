#!/bin/bash
# The N-rank bench path (torchrun, StepBoard, node-shared record slots, rank
# 0's merge in global unit order) end to end on a one-GPU box: every rank on
# device 0 (UNIPEAK_SHARE_GPU), gloo for the setup collectives (RCCL refuses
# two ranks on one GPU).  The merged region counts must equal N=1's.
R="${GRAFT_REPO_ROOT:?}"; cd "$R" || exit 1; mkdir -p gpurun_out/rehearse
for N in ${NS:-2 4}; do
  UNIPEAK_SHARE_GPU=1 UNIPEAK_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 20 \
    --warmup 3 --no-cpu-baseline > gpurun_out/rehearse/n$N.json 2> gpurun_out/rehearse/n$N.err || { tail -20 gpurun_out/rehearse/n$N.err; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['value'], d['ms_per_step'], d['regions'])" gpurun_out/rehearse/n$N.json $N
done
