#!/usr/bin/env python3
"""Does the HIP runtime bundled with torch coexist with the system HIP runtime
our library links?  Runs each order in a fresh subprocess."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

BODY = {
    "torch_first": """
import torch
torch.cuda.set_device(0)
x = torch.ones(4, device='cuda:0'); torch.cuda.synchronize()
from unipeak_amd import capi
with capi.Lib(0) as g:
    g.set_params(50, 1, 0.003); u = g.add_unit(100000); g.synth(u, 0, 0, 1, 0, 0, False, True)
    n = g.run()
print('OK torch_first', n, float(x.sum()))
""",
    "lib_first": """
from unipeak_amd import capi
with capi.Lib(0) as g:
    g.set_params(50, 1, 0.003); u = g.add_unit(100000); g.synth(u, 0, 0, 1, 0, 0, False, True)
    n = g.run()
import torch
x = torch.ones(4, device='cuda:0'); torch.cuda.synchronize()
print('OK lib_first', n, float(x.sum()))
""",
    "torch_dist_first": """
import os, torch, torch.distributed as dist
os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT='29533', RANK='0', WORLD_SIZE='1')
torch.cuda.set_device(0)
dist.init_process_group('nccl')
t = torch.ones(1, device='cuda:0'); dist.all_reduce(t)
from unipeak_amd import capi
with capi.Lib(0) as g:
    g.set_params(50, 1, 0.003); u = g.add_unit(100000); g.synth(u, 0, 0, 1, 0, 0, False, True)
    n = g.run()
dist.all_reduce(t); torch.cuda.synchronize()
print('OK torch_dist_first', n, float(t.item()))
dist.destroy_process_group()
""",
}

for name, body in BODY.items():
    r = subprocess.run([sys.executable, "-c", body], cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    tail = (r.stdout + r.stderr).strip().splitlines()[-3:]
    print(f"{name}: rc={r.returncode} :: " + " | ".join(tail), flush=True)
