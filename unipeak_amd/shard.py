"""unipeak_amd/shard.py -- multi-GPU layout of the region scan.

A ProfileBuffer's state is reset by flushContig() (misc/peakcall.cpp:224-231),
so one (contig, buffer) pass -- a *unit* -- is independent of every other
unit once the global background is known.  The only cross-GPU data the
reference's computation needs is the pooled tag total behind the background
density (src/regions.cpp:205-213); the region records then travel to rank 0.
So the layout is:

* ``plan()``      -- LPT of units over ranks by track bytes (no unit is split);
* ``Comm.global_tags()``  -- ONE all-reduce (RCCL over xGMI on GPUs, gloo on CPU);
* ``Comm.gather_records()`` -- one max-count all-reduce + one gather of the
  fixed-size records to rank 0 (RCCL when the ranks own GPUs);
* ``merge()``     -- rank 0 concatenates the per-rank, unit-major record
  blocks in global unit order (a slice per unit, no sort).

Units of one rank are run in ascending global order, so each rank's records
are already unit-major; the CLI engine (host/engine.cpp) applies the same
plan inside one process over several devices and then restores the
reference's emission order from the replayed event clock.
"""
from __future__ import annotations

import numpy as np


def units_for(contig_lens, nondir):
    """Units in the reference's pass order: directional runs feed a forward
    and a reverse ProfileBuffer (src/regions.cpp:331-356) -- unit (contig, 0)
    for the forward buffer and (contig, 1) for the reverse one; nondirectional
    runs feed one buffer with both strands (unit (contig, 0))."""
    n = len(contig_lens)
    if nondir:
        return [(ci, 0) for ci in range(n)]
    return [(ci, b) for b in (0, 1) for ci in range(n)]


def lpt(weights, world):
    """Longest-processing-time assignment: heaviest unit first onto the least
    loaded rank (ties -> lowest rank, so every rank computes the same plan)."""
    order = sorted(range(len(weights)), key=lambda i: (-weights[i], i))
    load = [0] * world
    owner = [0] * len(weights)
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        owner[i] = r
        load[r] += weights[i]
    return owner, load


def plan(contig_lens, nondir, world, n_samples=1):
    """-> (units, owner, per-rank unit lists in ascending global order)."""
    units = units_for(contig_lens, nondir)
    nstr = 2 if nondir else 1
    weights = [int(contig_lens[ci]) * nstr * n_samples * 4 for ci, _ in units]
    owner, _ = lpt(weights, world)
    mine = [[k for k in range(len(units)) if owner[k] == r] for r in range(world)]
    return units, owner, mine


def merge(parts, n_units, dtype):
    """parts: [(records, local->global unit ids, counts or None)] from every
    rank, each unit-major.  Returns (records, global unit id per record,
    counts) in global unit order."""
    if len(parts) == 1:
        recs, gids, cnt = parts[0]
        gids = np.asarray(gids, np.int64)
        if np.all(gids[1:] > gids[:-1]):  # one rank, units already in global order
            return recs, gids[recs["unit"].astype(np.int64)], cnt
    blocks = []
    for recs, gids, cnt in parts:
        gids = np.asarray(gids, np.int64)
        if len(recs) == 0:
            continue
        loc = recs["unit"].astype(np.int64)
        bounds = np.searchsorted(loc, np.arange(len(gids) + 1), side="left")
        for li, g in enumerate(gids):
            a, b = int(bounds[li]), int(bounds[li + 1])
            if b > a:
                blocks.append((int(g), recs[a:b], None if cnt is None else cnt[a:b]))
    blocks.sort(key=lambda t: t[0])
    if not blocks:
        return np.zeros(0, dtype), np.zeros(0, np.int64), None
    recs = np.concatenate([b[1] for b in blocks])
    gid = np.concatenate([np.full(len(b[1]), b[0], np.int64) for b in blocks])
    cnt = None if blocks[0][2] is None else np.concatenate([b[2] for b in blocks])
    return recs, gid, cnt


class Comm:
    """torch.distributed plumbing for the two exchanges of a step.

    ``device`` is ``"cuda:<local>"`` when the default group is RCCL (backend
    "nccl" on ROCm) and ``"cpu"`` for gloo; the collectives and their order
    are the same either way, which is what the gloo tests exercise."""

    def __init__(self, dist, rank, world, device):
        import torch
        self.torch = torch
        self.dist = dist
        self.rank = rank
        self.world = world
        self.device = device

    def global_tags(self, local_tags: int) -> int:
        """The single data-path collective of the scan (regions.cpp:205-213)."""
        t = self.torch.tensor([int(local_tags)], dtype=self.torch.int64, device=self.device)
        self.dist.all_reduce(t)
        return int(t.item())

    def max_over_ranks(self, x: float) -> float:
        t = self.torch.tensor([float(x)], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, x: float) -> float:
        t = self.torch.tensor([float(x)], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t)
        return float(t.item())

    def gather_records(self, recs: np.ndarray, extra: np.ndarray | None = None):
        """Fixed-size records (+ an optional fixed-width uint32 row per record)
        to rank 0.  Returns a list of (records, extra) per rank on rank 0,
        None elsewhere."""
        torch = self.torch
        n = len(recs)
        nmax = int(self.max_over_ranks(n))
        rb = recs.dtype.itemsize
        eb = 0 if extra is None else extra.shape[1] * 4
        row = rb + eb
        buf = np.zeros((max(nmax, 1), row + 8), np.uint8)
        buf[:n, :rb] = recs.view(np.uint8).reshape(n, rb)
        if eb:
            buf[:n, rb:rb + eb] = np.ascontiguousarray(extra, np.uint32).view(np.uint8).reshape(n, eb)
        buf[0, row:row + 8] = np.frombuffer(np.int64(n).tobytes(), np.uint8)
        t = torch.from_numpy(buf).to(self.device)
        glist = [torch.empty_like(t) for _ in range(self.world)] if self.rank == 0 else None
        self.dist.gather(t, glist, dst=0)
        if self.rank != 0:
            return None
        out = []
        for g in glist:
            a = g.cpu().numpy()
            k = int(np.frombuffer(a[0, row:row + 8].tobytes(), np.int64)[0])
            r = np.ascontiguousarray(a[:k, :rb]).view(recs.dtype).reshape(k)
            e = None if not eb else np.ascontiguousarray(a[:k, rb:rb + eb]).view(np.uint32).reshape(k, -1)
            out.append((r, e))
        return out
