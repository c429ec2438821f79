"""x-slab decomposition of the SPH step over ranks.

The reference runs one FluidSystem on one device (fluid.cpp:958-1021); here
the particle set is split by x into one slab per rank and every rank runs
the same lpe_sph_step / lpe_world_tick on the particles it owns, exchanging
the particles within two reference-cell columns of its edges with its two
neighbours every sub-step (include/lpe.h, "x-slab decomposition").  A rank
owns the particles whose reference-cell column floor((x + eps) / 2h) lies in
its slab, decided anew from every sub-step's kicked position, so a particle
that crosses an edge changes owner inside that sub-step.  This module holds
the host side of that split:

  slab_edges      equal-count slab edges on reference-cell boundaries
  owners          owning rank of each particle (the device's cell-column rule)
  wire_capacity   ghost records per direction and sub-step
  setup_rank      configure + upload one rank's context
  merge_owned     reassemble the global state from the ranks' owned sets
  broadcast_uid / gather_owned   the torch.distributed plumbing (RCCL id
                  exchange, gather of the owned sets to rank 0)

Nothing here runs a physics kernel; the device work is all behind the C ABI.
"""
from __future__ import annotations

import numpy as np

FIELDS = ("x", "y", "vx", "vy", "density", "pressure")
BAND = 2                  # ghost cell columns each side of an edge (lpe_sph.hip SLAB_BAND)
BAND_CAP = 3              # ... in the reference cell-capacity mode: at least (SLAB_BAND_CAP), one more per
BAND_MAX = 8              #   65 particles the largest cell holds past 64, at most SLAB_BAND_MAX
BAND_CAP_WIRE = 5         # the capped mode's default wire: cells of up to 194 (lpe_sph.hip slab_band)


def cell_size(cfg=None) -> float:
    """The reference cell size 2 max(0.05, h) (fluid.cpp:724-737), fp32."""
    h = 0.05 if cfg is None else float(cfg.gridConfig.smoothingLength)
    return float(np.float32(2.0) * np.float32(max(0.05, h)))


def _columns(x, cfg=None):
    """Reference-cell column of each x: floor((x + eps) / cs) in fp32, the
    device's bin column (lpe_sph.hip bin_key)."""
    eps = np.float32(1e-6 if cfg is None else cfg.gridConfig.gridEpsilon)
    cs = np.float32(cell_size(cfg))
    return np.floor((np.asarray(x, np.float32) + eps) / cs).astype(np.int64)


def slab_edges(x, nranks: int, cfg=None) -> np.ndarray:
    """nranks + 1 float32 edges [-inf, e1, ..., e_{n-1}, +inf]: inner edges on
    reference-cell boundaries at the column-count quantiles of the particles
    (every slab starts with ~N/nranks particles), at least 8 columns apart.
    Deterministic in x, so every rank computes the same edges."""
    cs = cell_size(cfg)
    col = np.sort(_columns(x, cfg))
    n = len(col)
    cuts = []
    for r in range(1, nranks):
        c = int(col[min(n - 1, (n * r) // nranks)]) if n else 8 * r
        if cuts and c < cuts[-1] + 8:
            c = cuts[-1] + 8
        cuts.append(c)
    edges = [np.float32(-np.inf)] + [np.float32(c * cs) for c in cuts] + [np.float32(np.inf)]
    return np.array(edges, np.float32)


def owners(x, edges, cfg=None) -> np.ndarray:
    """Owning rank of each particle: slab r holds the particles whose cell
    column lies in [edges[r] / cs, edges[r+1] / cs) (the device's rule)."""
    cs = cell_size(cfg)
    cuts = np.rint(np.asarray(edges, np.float64)[1:-1] / cs).astype(np.int64)
    return np.searchsorted(cuts, _columns(x, cfg), side="right").astype(np.int32)


def wire_capacity(x, edges, cfg=None, factor: float = 2.0, floor: int = 2048, band: int = BAND) -> int:
    """Ghost records per direction and sub-step: `factor` times the most
    particles in the band + 1 columns along any inner edge at the start (the
    band, a column the re-balancing may move, room for compression), plus
    `floor`."""
    BAND = band
    col = _columns(x, cfg)
    cs = cell_size(cfg)
    worst = 0
    for e in np.asarray(edges, np.float64)[1:-1]:
        c = int(round(e / cs))
        worst = max(worst, int(((col >= c - BAND - 1) & (col < c)).sum()),
                    int(((col >= c) & (col < c + BAND + 1)).sum()))
    return int(factor * worst) + floor


def setup_rank(ctx, rank: int, nranks: int, fluid: dict, edges, cfg, rigids=None, wire_cap=None,
               domain=None, rebalance: int = 0, cells: str = "unbounded"):
    """Configure ctx as slab `rank` and upload the particles it owns (global
    ids = indices into `fluid`).  cells="ref": the reference's 64-particle
    cells (LPE_SPH_MODE_REF_CELL_CAP; the global count and a wire for
    BAND_CAP ghost columns).  Returns the owned global ids."""
    import lpe  # the in-tree binding (little-physics-engine_amd/lpe.py)
    x = np.asarray(fluid["x"], np.float32)
    if wire_cap is None:
        wire_cap = wire_capacity(x, edges, cfg, band=BAND_CAP_WIRE if cells == "ref" else BAND)
    own = np.nonzero(owners(x, edges, cfg) == rank)[0].astype(np.int32)
    ctx.sph_set_config(cfg)
    ctx.sph_set_slab(nranks, rank, edges, wire_cap, rebalance)
    sub = {k: np.asarray(fluid[k])[own] for k in ("x", "y", "vx", "vy", "mass", "density", "pressure")}
    ctx.sph_upload(sub["x"], sub["y"], sub["vx"], sub["vy"], sub["mass"], sub["density"], sub["pressure"])
    ctx.sph_set_ids(own)
    if cells == "ref":
        ctx.sph_set_global_count(len(x))
        ctx.sph_set_mode(lpe.SPH_MODE_REF_CELL_CAP)
    if domain is None:
        y = np.asarray(fluid["y"], np.float32)
        pad = 1.0
        domain = (float(x.min()) - pad, float(y.min()) - pad, float(x.max()) + pad, float(y.max()) + pad)
    ctx.sph_set_domain(*domain)
    ctx.sph_upload_rigids(rigids if rigids is not None else np.zeros(0, lpe.RIGID_DTYPE))
    return own


def rebalance_edges(hist, col0: int, edges, edges0, nranks: int, mv: int, minw: int = 8):
    """One re-balancing move, as k_slab_rebalance (lpe_sph.hip) does it on the
    device from the all-reduced column histogram: each inner edge j moves one
    column towards the j / nranks count quantile unless the particles left
    of it are within max(1 % of a slab's mean, half its column) of the
    target, stays within edges0[j] -/+ mv and minw columns of its
    neighbours.  fp32 sums as the device's (counts are exact integers)."""
    hist = np.asarray(hist, np.float32)
    e = np.array(edges, np.int64)
    total = np.float32(hist.sum(dtype=np.float64))
    for j in range(1, nranks):
        c = int(e[j]) - col0
        left = np.float32(hist[:max(0, min(c, len(hist)))].sum(dtype=np.float64))
        target = np.float32(total * np.float32(j) / np.float32(nranks))
        colc = np.float32(hist[c]) if 0 <= c < len(hist) else np.float32(0.0)
        tol = max(np.float32(0.01) * total / np.float32(nranks), np.float32(0.5) * colc)
        ne = int(e[j])
        if left < target - tol:
            ne += 1
        elif left > target + tol:
            ne -= 1
        ne = min(max(ne, int(edges0[j]) - mv), int(edges0[j]) + mv)
        if j > 1:
            ne = max(ne, int(e[j - 1]) + minw)
        if j + 1 < nranks:
            ne = min(ne, int(e[j + 1]) - minw)
        e[j] = ne
    return e


def merge_owned(parts, n_global: int) -> dict:
    """Global arrays (index = global id) from the ranks' owned sets; every id
    must appear exactly once."""
    out = {k: np.zeros(n_global, np.float32) for k in FIELDS}
    seen = np.zeros(n_global, np.int32)
    for p in parts:
        ids = np.asarray(p["id"], np.int64)
        if len(ids) and (ids.min() < 0 or ids.max() >= n_global):
            raise ValueError("slab merge: particle id out of range")
        np.add.at(seen, ids, 1)
        for k in FIELDS:
            out[k][ids] = p[k]
    if not (seen == 1).all():
        lost, dup = int((seen == 0).sum()), int((seen > 1).sum())
        raise ValueError(f"slab merge: {lost} particles lost, {dup} duplicated")
    return out


# ---- torch.distributed plumbing (one process per GPU) ---------------------
def broadcast_uid(uid: bytes | None, rank: int) -> bytes:
    """Rank 0's 128-byte RCCL id to every rank (over the default process
    group: gloo or nccl)."""
    import torch.distributed as dist
    box = [uid if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    return box[0]


def gather_owned(owned: dict, n_global: int, rank: int, world: int):
    """The merged global state on rank 0 (None on the others)."""
    import torch.distributed as dist
    parts = [None] * world if rank == 0 else None
    dist.gather_object({k: np.asarray(v) for k, v in owned.items()}, parts, dst=0)
    return merge_owned(parts, n_global) if rank == 0 else None


class GlooTransport:
    """The host-staged slab transport (lpe_mg_init_host) over the default
    torch.distributed process group (gloo): the cross-process counterpart of
    the in-process loopback, for validating the exchange protocol where RCCL
    cannot run (two ranks on one GPU).  Every halo first swaps a 2-word header
    per link, [bytes I send you, bytes I expect from you], so both ends see
    the same four sizes and a mismatch fails on both ends instead of hanging
    or truncating; then the payloads move with isend / irecv."""

    def __init__(self, rank: int, world: int):
        self.rank, self.world = rank, world
        self.last_error = None
        self.calls = {"halo": 0, "allreduce_f32": 0, "allreduce_i64": 0}

    def halo(self, sendL, sendR, recvL, recvR):
        import torch
        import torch.distributed as dist
        self.calls["halo"] += 1
        links = []
        if self.rank > 0 and sendL is not None:
            links.append((self.rank - 1, sendL, recvL))
        if self.rank < self.world - 1 and sendR is not None:
            links.append((self.rank + 1, sendR, recvR))
        hdr_out, hdr_in, reqs = [], [], []
        for peer, s, r in links:
            mine = torch.tensor([s.nbytes, 0 if r is None else r.nbytes], dtype=torch.int64)
            theirs = torch.zeros(2, dtype=torch.int64)
            hdr_out.append(mine)
            hdr_in.append(theirs)
            reqs += [dist.isend(mine, peer), dist.irecv(theirs, peer)]
        for q in reqs:
            q.wait()
        bad = [peer for (peer, _, _), m, t in zip(links, hdr_out, hdr_in)
               if int(t[0]) != int(m[1]) or int(t[1]) != int(m[0])]
        if bad:
            raise RuntimeError(f"slab halo: rank {self.rank}: send/receive sizes differ from rank(s) {bad}'s "
                               f"({[(m.tolist(), t.tolist()) for m, t in zip(hdr_out, hdr_in)]})")
        reqs = []
        for peer, s, r in links:
            reqs.append(dist.isend(torch.from_numpy(s), peer))
            if r is not None:
                reqs.append(dist.irecv(torch.from_numpy(r), peer))
        for q in reqs:
            q.wait()

    def allreduce_f32(self, arr, op):
        import torch
        import torch.distributed as dist
        self.calls["allreduce_f32"] += 1
        dist.all_reduce(torch.from_numpy(arr), op=dist.ReduceOp.MIN if op else dist.ReduceOp.SUM)

    def allreduce_i64(self, arr):
        import torch
        import torch.distributed as dist
        self.calls["allreduce_i64"] += 1
        dist.all_reduce(torch.from_numpy(arr), op=dist.ReduceOp.SUM)
