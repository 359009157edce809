#!/usr/bin/env python3
"""Headline benchmark: genome Gbp/s for KDE smoothing + region scan on hg19.

Default workload (BASELINE.json configs[1], the metric's config): hg19 full
genome (25 contigs, 3,095,693,983 bp), one directional sample (3SEQ-style),
default parameters (bw 50, -r 25, -k 50, -t 10), synthetic hg19-shaped tag
counts generated on the device, packed to uint8 tracks and
resident in HBM before timing.  Other BASELINE configs are available with
--workload for our own measurements (the default line is the headline):

  hg19-dir1    configs[1]  1 directional sample                      (default)
  hg19-nondir1 configs[2]  regions pass of C3: -D -y, 1 sample, both strands
  hg19-8s1c    configs[3]  8 samples + 1 negative control (-e 9), directional
  hg19mm9-32s  configs[4]  hg19+mm9, 32 samples, -D -k 50 -u 0.3 -y (8 GPUs)

One step = the whole hot path over the genome: RCCL all-reduce of the tag
totals -> background -> up_run (K1a stream+screen -> K1b exact blocks -> K2
segmentation -> K3 region statistics + filters, one stream, records written
straight into pinned host memory) -> (N>1) RCCL gather of the records to
rank 0 -> records in global unit order.

Multi-GPU: one process per GPU (torchrun); units are LPT-assigned to ranks by
unipeak_amd/shard.py (strong scaling: the genome is fixed), so there is no
data-path collective besides the RCCL background all-reduce and the record
gather.  UNIPEAK_BENCH_DIST=1 takes the distributed path at N=1 too (to
exercise RCCL on a one-GPU box).

Prints ONE JSON line on rank 0 (contract in the task statement), including
the roofline of the dominant kernel (K1a) and the oracle CPU baseline.
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

WORKLOADS = {
    "hg19-dir1": dict(tables=["hg19"], nondir=False, samples=1, controls=0, kurt=50.0, corr=-1.0,
                      want_corr=False, baseline="configs[1]",
                      desc="hg19 full genome, 1 directional sample (3SEQ-style), bw 50, "
                           "-r 25 -k 50 -t 10 (BASELINE configs[1])"),
    "hg19-nondir1": dict(tables=["hg19"], nondir=True, samples=1, controls=0, kurt=50.0, corr=-1.0,
                         want_corr=True, baseline="configs[2]",
                         desc="hg19, 1 nondirectional sample, regions -D -y pass of C3, bw 50, "
                              "-r 25 -k 50 -t 10 (BASELINE configs[2])"),
    "hg19-8s1c": dict(tables=["hg19"], nondir=False, samples=9, controls=1, kurt=50.0, corr=-1.0,
                      want_corr=False, baseline="configs[3]",
                      desc="hg19, 8 pooled directional samples + 1 negative control (-e 9), bw 50, "
                           "-r 25 -k 50 -t 10 (BASELINE configs[3])"),
    "hg19mm9-32s": dict(tables=["hg19", "mm9"], nondir=True, samples=32, controls=0, kurt=50.0,
                        corr=0.3, want_corr=True, baseline="configs[4]",
                        desc="hg19+mm9 (names prefixed), 32 nondirectional samples, -D -k 50 -u 0.3 -y, "
                             "bw 50 (BASELINE configs[4])"),
}


def read_contigs(path):
    out = []
    for line in open(path):
        f = line.split()
        if len(f) >= 2 and not line.startswith("#"):
            out.append((f[0], int(f[1])))
    return out


def load_table(names):
    contigs = []
    for t in names:
        rows = read_contigs(os.path.join(ROOT, "unipeak_amd", "data", f"{t}.txt"))
        contigs += [((f"{t}_{n}" if len(names) > 1 else n), L) for n, L in rows]
    return contigs


def pmc_traffic(bytes_per_launch):
    """HBM bytes per K1a launch from the committed rocprofv3 PMC passes
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
    ap.add_argument("--workload", default="hg19-dir1", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", default="all")
    args = ap.parse_args()
    W = WORKLOADS[args.workload]

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    comm = None
    if world > 1 or os.environ.get("UNIPEAK_BENCH_DIST") == "1":
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)  # torch's HIP runtime first (tools/mix_probe.py)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29577")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
        dist.init_process_group("nccl")  # RCCL over xGMI
        comm = shard.Comm(dist, rank, world, f"cuda:{local}")

    contigs = load_table(W["tables"])
    genome = sum(L for _, L in contigs)
    mappable = genome & 0xFFFFFFFF  # ContigTable::genomeSize_ is uint32 (quirk Q10)
    lens = [L for _, L in contigs]
    S, n_ctl, nondir = W["samples"], W["controls"], W["nondir"]
    s_nc = S - n_ctl
    nstr = 2 if nondir else 1
    units, owner, mine_all = shard.plan(lens, nondir=nondir, world=world, n_samples=S)
    mine = mine_all[rank]
    need = sum(lens[units[k][0]] * nstr * S for k in mine)
    if need > 250e9:
        raise SystemExit(f"workload {args.workload} needs {need / 1e9:.0f} GB of tracks per GPU at "
                         f"N={world}; run it on more GPUs")

    control = [0] * s_nc + [1] * n_ctl
    g = capi.Lib(local)
    g.set_params(args.bw, S, 0.0029, nondir=nondir, control=control)  # background set per step
    t_gen = time.time()
    for k in mine:  # ascending global order: records come back unit-major
        ci, buf = units[k]
        u = g.add_unit(lens[ci], buffer_id=buf)
        for st in range(nstr):
            synth_strand = st if nondir else buf
            for smp in range(S):
                seed = args.seed + smp if smp < s_nc else 2000 + (smp - s_nc)
                g.synth(u, st, smp, seed, ci, synth_strand, nondir=nondir, peaks=smp < s_nc)
    local_tags = sum(g.tag_total(i, st, smp) for i in range(len(mine)) for st in range(nstr)
                     for smp in range(s_nc))
    gen_s = time.time() - t_gen
    # K1a algorithmic bytes: one uint8 count per bp per strand per non-control
    # sample
    alg_bytes = sum(lens[units[k][0]] * nstr * s_nc for k in mine)
    copy_gbps = g.hbm_copy_gbps(1 << 30, 5)

    phase = {"allreduce": 0.0, "run": 0.0, "gather_merge": 0.0}
    # one node (torchrun --nnodes=1): records meet in node-shared host memory
    gather_mode = os.environ.get("UNIPEAK_GATHER") or (
        "shm" if int(os.environ.get("LOCAL_WORLD_SIZE", world)) == world else "rccl")
    bg_set = [None]
    nr = rbuf = cap = None
    pool = pending = None
    # size the record slots once (the data are the same every step): one
    # untimed pass with host delivery, then K3 writes every later pass
    # straight into the slots, and rank 0 reads step i-1's slots on a helper
    # thread while step i runs (up_run releases the GIL)
    g.set_params(args.bw, S, (comm.global_tags(local_tags) if comm else local_tags) / mappable /
                 (1 if nondir else 2), region_thr=25.0, kurt_thr=W["kurt"], corr_thr=W["corr"],
                 hit_thr=10.0 * s_nc, nondir=nondir, control=control, want_corr=W["want_corr"])
    n0 = g.run()
    cap = int((comm.max_over_ranks(n0) if comm else n0) * 1.25) + 64
    if comm is None or gather_mode == "shm":
        tag = f"{os.environ.get('TORCHELASTIC_RUN_ID', 'run')}_{os.environ.get('MASTER_PORT', '0')}"
        nr = shard.NodeRecords(comm, cap, S, capi.REGION_DTYPE.itemsize, tag)
        g.host_register(*nr.my_range())
        if rank == 0:
            from concurrent.futures import ThreadPoolExecutor
            pool = ThreadPoolExecutor(1)
    else:
            rbuf = comm.target_buffer(cap, S, capi.REGION_DTYPE.itemsize)
            comm.torch.cuda.synchronize()
            g.set_record_target(rbuf.data_ptr(), cap)
    it = [0]

    def consume(parts):
        """rank 0: every rank's records in global unit order (zero-copy blocks)"""
        blocks = shard.order_blocks([(r, mine_all[i], e) for i, (r, e) in enumerate(parts)])
        return (sum(len(b[1]) for b in blocks),
                sum(int(np.count_nonzero(b[1]["accepted"])) for b in blocks))

    def step():
        nonlocal pending
        t0 = time.perf_counter()
        res = None
        if pending is not None:  # step i-2's slots are free again once rank 0 read them
            res = pending.result()
            pending = None
        tags = comm.global_tags(local_tags) if comm else local_tags
        if nr is not None and rank == 0 and it[0] > 0:
            # every rank entered this step, so step i-1 is in its slots: read it
            # while this step runs (up_run releases the GIL)
            pending = pool.submit(lambda p=(it[0] - 1) & 1: consume(nr.read(capi.REGION_DTYPE, p)))
        # regions.cpp:205-213: tags / mappable, per strand when directional
        background = tags / mappable / (1 if nondir else 2)
        if bg_set[0] != background:
            g.set_params(args.bw, S, background, region_thr=25.0, kurt_thr=W["kurt"],
                         corr_thr=W["corr"], hit_thr=10.0 * s_nc, nondir=nondir, control=control,
                         want_corr=W["want_corr"])
            bg_set[0] = background
        if nr is not None:
            g.set_record_target(nr.my_slot_address(it[0] & 1), cap)
        t1 = time.perf_counter()
        n = g.run()
        t2 = time.perf_counter()
        if rbuf is not None:  # RCCL gather of the device record buffers
            raw = comm.gather_target(rbuf)
            if raw is not None:
                res = consume([shard.parse_target(raw[i], cap, S, capi.REGION_DTYPE) for i in range(world)])
        it[0] += 1
        t3 = time.perf_counter()
        phase["allreduce"] += t1 - t0
        phase["run"] += t2 - t1
        phase["gather_merge"] += t3 - t2
        return n, res, g.timings()

    def drain():
        """the last step's records (shm: after every rank finished it)"""
        nonlocal pending
        if nr is None:
            return None
        res = None
        if pending is not None:
            res = pending.result()
            pending = None
        if comm is not None:
            comm.dist.barrier()
        if rank == 0:
            res = consume(nr.read(capi.REGION_DTYPE, (it[0] - 1) & 1))
        return res

    def barrier():
        if comm is not None:
            comm.dist.barrier()

    for _ in range(args.warmup):
        st = step()
        if rank == 0:
            tt = st[2]
            print(f"[bench] warmup: K1 {tt[0]:.3f} ms (exact part {tt[4]:.3f}), K2 {tt[1]:.3f} ms, "
                  f"K3 {tt[2]:.3f} ms, up_run wall {tt[3]:.3f} ms", file=sys.stderr, flush=True)
    drain()
    for k in phase:
        phase[k] = 0.0
    barrier()
    if comm is not None:
        comm.torch.cuda.synchronize()
    t0 = time.perf_counter()
    k1, k1a = [], []
    last = None
    for _ in range(args.steps):
        last = step()
        k1.append(last[2][0])
        k1a.append(last[2][0] - last[2][4])  # K1a = K1 minus its exact part (K1b)
    final = drain()  # inside the timed region: the last step's records reach rank 0
    if final is not None:
        last = (last[0], final, last[2])
    barrier()
    if comm is not None:
        comm.torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    k1_ms = float(np.mean(k1))
    k1a_ms = float(np.mean(k1a))
    my_achieved = alg_bytes / (k1a_ms * 1e-3) / 1e9
    if comm is not None:
        dt = comm.max_over_ranks(dt)
        achieved = comm.sum_over_ranks(my_achieved) / world  # mean per-GPU K1a GB/s
        k1a_max = comm.max_over_ranks(k1a_ms)
    else:
        achieved, k1a_max = my_achieved, k1a_ms

    if rank == 0:
        print("[bench] per-step phases (ms): " + ", ".join(
            f"{k} {v / args.steps * 1e3:.3f}" for k, v in phase.items()), file=sys.stderr, flush=True)
        value = genome / dt / 1e9
        traffic, traffic_src = (pmc_traffic(alg_bytes) if (world == 1 and args.workload == "hg19-dir1")
                                else (None, None))
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
            "config": {"workload": W["desc"], "baseline_config": W["baseline"],
                       "genome_bp": genome, "units": len(units), "samples": S,
                       "parallelism": f"contig{'' if nondir else '-strand'} units LPT over {world} GPU(s)"},
            "regions": {"candidates": int(last[1][0]), "accepted": int(last[1][1])},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "traffic_unit": "GB per launch (rocprofv3 PMC FETCH_SIZE+WRITE_SIZE, gfx950-corrected)",
                         "traffic_source": traffic_src,
                         "kernel": "scan_kernel<..., kModeScreen> (K1a: stream + integer screen)",
                         "kernel_ms": round(k1a_ms, 4), "kernel_ms_max_rank": round(k1a_max, 4),
                         "bytes_per_launch": int(alg_bytes),
                         "bytes_rule": "1 B (uint8 count) per bp per strand per non-control sample",
                         "k1_total_ms": round(k1_ms, 4),
                         "k1b_exact_ms": round(k1_ms - k1a_ms, 4),
                         "hbm_copy_GBps": round(copy_gbps, 1),
                         "frac_of_copy_rate": round(achieved / copy_gbps, 4)},
            "setup_s": round(gen_s, 2),
        }
        if world == 1 and not args.no_cpu_baseline and args.workload == "hg19-dir1":
            res["cpu_baseline"] = cpu_baseline(contigs, args, value)
        print(json.dumps(res), flush=True)
    g.set_record_target(0, 0)
    g.close()
    if pool is not None:
        pool.shutdown()
    if comm is not None:
        comm.dist.barrier()
        if nr is not None:
            nr.close()
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
            "sample": f"hg19 {'full genome' if args.cpu_sample == 'all' else args.cpu_sample} synthetic, "
                      f"directional, 1 sample, both strands ({bp} bp), oracle ProfileBuffer restatement, "
                      f"hits pre-parsed",
            "gpu_over_cpu": round(gpu_value / (bp / sec / 1e9), 1)}


if __name__ == "__main__":
    main()
