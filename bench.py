#!/usr/bin/env python3
"""Headline benchmark: genome Gbp/s for KDE smoothing + region scan on hg19.

Workload (BASELINE.json configs[1]): hg19 full genome (25 contigs,
3,095,693,983 bp), one directional sample (3SEQ-style), default parameters
(bw 50, -r 25, -k 50, -t 10), synthetic hg19-shaped tag counts generated on
the device (DESIGN.md "Synthetic input"), already resident in HBM.

One step = the whole hot path over the genome: RCCL all-reduce of the tag
totals -> background -> K1 scan (pool + KDE + flags + run boundaries) ->
K2 segmentation -> K3 region statistics + filters -> region records on the
host (pinned) -> (N>1) gather of the records to rank 0 -> records concatenated
in global unit order.

Multi-GPU: one process per GPU (torchrun); the 50 (contig, strand) units are
LPT-assigned to ranks by unipeak_amd/shard.py (strong scaling: the genome is
fixed), so there is no data-path collective besides the RCCL background
all-reduce and the RCCL gather of the fixed-size region records to rank 0.

Prints ONE JSON line on rank 0 (contract in the task statement), including
the roofline of the dominant kernel (K1) and the oracle CPU baseline.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from unipeak_amd import capi, shard  # noqa: E402

METRIC = "genome Gbp/s for KDE smoothing + region scan on hg19, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def read_contigs(path):
    out = []
    for line in open(path):
        f = line.split()
        if len(f) >= 2 and not line.startswith("#"):
            out.append((f[0], int(f[1])))
    return out


def pmc_traffic(bytes_per_launch):
    """HBM bytes per K1 launch from the committed rocprofv3 PMC passes
    (tools/pmc_traffic.py) when they were taken on this exact workload."""
    p = os.path.join(ROOT, "profiles", "r01", "k1a_pmc_traffic.json")
    try:
        d = json.load(open(p))
    except (OSError, ValueError):
        return None, None
    if int(d.get("algorithmic_bytes_per_launch", -1)) != int(bytes_per_launch):
        return None, None
    return round(d["traffic_bytes_per_launch"] / 1e9, 3), os.path.relpath(p, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--bw", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", default="all")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    comm = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")  # RCCL over xGMI
        comm = shard.Comm(dist, rank, world, f"cuda:{local}")

    contigs = read_contigs(os.path.join(ROOT, "unipeak_amd", "data", "hg19.txt"))
    genome = sum(L for _, L in contigs)
    lens = [L for _, L in contigs]
    units, owner, mine_all = shard.plan(lens, nondir=False, world=world)
    mine = mine_all[rank]

    g = capi.Lib(local)
    g.set_params(args.bw, 1, 0.0029)  # background is replaced every step
    t_gen = time.time()
    for k in mine:  # ascending global order: records come back unit-major
        ci, st = units[k]
        u = g.add_unit(lens[ci], buffer_id=st)
        g.synth(u, 0, 0, args.seed, ci, st, nondir=False, peaks=True)
    local_tags = sum(g.tag_total(i, 0, 0) for i in range(len(mine)))
    gen_s = time.time() - t_gen
    # K1 algorithmic bytes: one uint8 count per bp per strand per non-control
    # sample
    alg_bytes = 1 * 1 * sum(lens[units[k][0]] for k in mine)

    phase = {"allreduce": 0.0, "run": 0.0, "gather_merge": 0.0}

    def step():
        t0 = time.perf_counter()
        tags = comm.global_tags(local_tags) if comm else local_tags
        background = tags / genome / 2  # directional: per strand (regions.cpp:205-213)
        g.set_params(args.bw, 1, background, region_thr=25.0, kurt_thr=50.0,
                     corr_thr=-1.0, hit_thr=10.0)
        t1 = time.perf_counter()
        n = g.run()
        regs, cnt = g.regions_view()
        t2 = time.perf_counter()
        res = None
        if comm is not None:
            parts = comm.gather_records(regs, cnt)
            if parts is not None:  # rank 0: records of every rank in global unit order
                parts = [(r, mine_all[i], e) for i, (r, e) in enumerate(parts)]
                recs, gid, _ = shard.merge(parts, len(units), capi.REGION_DTYPE)
                res = (len(recs), int(np.count_nonzero(recs["accepted"])))
        else:  # one rank: units were added in global order, records are unit-major
            res = (len(regs), int(np.count_nonzero(regs["accepted"])))
        t3 = time.perf_counter()
        phase["allreduce"] += t1 - t0
        phase["run"] += t2 - t1
        phase["gather_merge"] += t3 - t2
        return n, res, g.timings()

    def barrier():
        if comm is not None:
            comm.dist.barrier()

    for _ in range(args.warmup):
        st = step()
        if rank == 0:
            tt = st[2]
            print(f"[bench] warmup: K1 {tt[0]:.3f} ms (exact part {tt[4]:.3f}), K2 {tt[1]:.3f} ms, K3 {tt[2]:.3f} ms, "
                  f"up_run wall {tt[3]:.3f} ms", file=sys.stderr, flush=True)
    for k in phase:
        phase[k] = 0.0
    barrier()
    t0 = time.perf_counter()
    k1 = []
    k1a = []
    last = None
    for _ in range(args.steps):
        last = step()
        k1.append(last[2][0])
        k1a.append(last[2][0] - last[2][4])  # K1a = K1 minus its exact part (K1b)
    barrier()
    dt = (time.perf_counter() - t0) / args.steps
    k1_ms = float(np.mean(k1))
    k1a_ms = float(np.mean(k1a))
    my_achieved = alg_bytes / (k1a_ms * 1e-3) / 1e9
    if comm is not None:
        dt = comm.max_over_ranks(dt)
        achieved = comm.sum_over_ranks(my_achieved) / world  # mean per-GPU K1 GB/s
        k1_max = comm.max_over_ranks(k1a_ms)
    else:
        achieved, k1_max = my_achieved, k1a_ms

    if rank == 0:
        print("[bench] per-step phases (ms): " + ", ".join(
            f"{k} {v / args.steps * 1e3:.3f}" for k, v in phase.items()), file=sys.stderr, flush=True)
        value = genome / dt / 1e9
        traffic, traffic_src = pmc_traffic(alg_bytes) if world == 1 else (None, None)
        res = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Gbp/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (device-generated hg19-shaped tag counts, DESIGN.md §8)",
            "config": {"workload": "hg19 full genome, 1 directional sample (3SEQ-style), "
                                   "bw 50, -r 25 -k 50 -t 10 (BASELINE configs[1])",
                       "genome_bp": genome, "units": len(units),
                       "parallelism": f"contig-strand units LPT over {world} GPU(s)"},
            "regions": {"candidates": int(last[1][0]), "accepted": int(last[1][1])},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_unit": "GB per launch (rocprofv3 PMC FETCH_SIZE+WRITE_SIZE, gfx950-corrected)",
                         "traffic_source": traffic_src,
                         "kernel": "scan_kernel<..., kModeScreen> (K1a: stream + integer screen)",
                         "kernel_ms": round(k1a_ms, 4), "kernel_ms_max_rank": round(k1_max, 4),
                         "bytes_per_launch": int(alg_bytes),
                         "bytes_rule": "1 B (uint8 count) per bp per strand per non-control sample",
                         "k1_total_ms": round(k1_ms, 4),
                         "k1b_exact_ms": round(k1_ms - k1a_ms, 4)},
            "setup_s": round(gen_s, 2),
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(contigs, args, value)
        print(json.dumps(res), flush=True)
    g.close()
    if comm is not None:
        comm.dist.destroy_process_group()


def cpu_baseline(contigs, args, gpu_value):
    """Oracle (plain-C restatement of ProfileBuffer) on 1 core over a bounded
    sample of the same synthetic genome, hot path only (hits pre-parsed)."""
    from tests.oracle_binding import Oracle
    orc = Oracle()
    names = [n for n, _ in contigs] if args.cpu_sample == "all" else args.cpu_sample.split(",")
    idx = [i for i, (n, _) in enumerate(contigs) if n in names]
    # the sample's contigs keep their hg19 contig indices for the generator:
    # pass lengths padded with zeros for skipped contigs
    lens = np.zeros(max(idx) + 1, np.uint32)
    for i in idx:
        lens[i] = contigs[i][1]
    genome = sum(L for _, L in contigs)
    bg = 22_600_000 / genome / 2  # fixed (hot path cost does not depend on it)
    npass, nrej, sec = orc.baseline(lens, args.seed, args.bw, 25.0, 50.0, 10.0, bg)
    bp = int(lens.sum())
    return {"value": round(bp / sec / 1e9, 4), "unit": "Gbp/s", "cores": 1, "kind": "port",
            "seconds": round(sec, 2),
            "sample": f"hg19 {'full genome' if args.cpu_sample == 'all' else args.cpu_sample} synthetic, directional, 1 sample, both "
                      f"strands ({bp} bp), oracle ProfileBuffer restatement, hits pre-parsed",
            "gpu_over_cpu": round(gpu_value / (bp / sec / 1e9), 1)}


if __name__ == "__main__":
    main()
