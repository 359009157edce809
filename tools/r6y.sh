#!/bin/bash
# is the slow cold leg the previous process's freed VRAM being reclaimed? a process fills 150 GB and exits,
# then the cold leg at once, then again after 40 s
R=$GRAFT_REPO_ROOT; F=$R/gpurun_out/r6y; mkdir -p $F
run() { tag=$1; UNIPEAK_BENCH_LEGS=cold UNIPEAK_BENCH_SINGLE=0 timeout -k 10 300 python $R/bench.py --no-cpu-baseline --steps 50 > $F/$tag.json 2> $F/$tag.err || { tail -3 $F/$tag.err; exit 1; }
  echo "$tag $(date +%s) $(grep 'cold:' $F/$tag.err | cut -c1-120)"; }
run before
timeout -k 10 120 python -c "
import torch, time
t = time.time()
x = [torch.ones(int(15e9) // 4, dtype=torch.int32, device='cuda') for _ in range(10)]
torch.cuda.synchronize(); print('filled 150 GB in', round(time.time() - t, 1), 's')
" || exit 1
echo "fill exited $(date +%s)"
run right_after
sleep 40
run after_40s
