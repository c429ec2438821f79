"""x-slab decomposition of the SPH step over ranks.

The reference runs one FluidSystem on one device (fluid.cpp:958-1021); here
the particle set is split by x into one slab per rank and every rank runs
the same lpe_sph_step on its owned particles, exchanging ghosts with its two
neighbours each sub-step (include/lpe.h, "x-slab decomposition").  This
module holds the host side of that split:

  slab_edges      equal-count slab edges (x-quantiles)
  owners          owning rank of each particle ([x0, x1) per slab)
  ghost_capacity  exchange-buffer size per side from the initial layout
  setup_rank      configure + upload one rank's context
  merge_owned     reassemble the global state from the ranks' owned sets
  broadcast_uid / gather_owned   the torch.distributed plumbing (RCCL id
                  exchange, gather of the owned sets to rank 0)

Nothing here runs a physics kernel; the device work is all behind the C ABI.
"""
from __future__ import annotations

import numpy as np

FIELDS = ("x", "y", "vx", "vy", "density", "pressure")


def slab_edges(x, nranks: int) -> np.ndarray:
    """nranks + 1 float32 edges [-inf, e1, ..., e_{n-1}, +inf]: inner edges at
    the x-quantiles of the particles, so every slab starts with ~N/nranks
    particles.  Deterministic in x, so every rank computes the same edges."""
    xs = np.sort(np.asarray(x, np.float32))
    n = len(xs)
    edges = [np.float32(-np.inf)]
    for r in range(1, nranks):
        e = xs[min(n - 1, (n * r) // nranks)] if n else np.float32(r)
        if e <= edges[-1]:
            e = np.nextafter(edges[-1], np.float32(np.inf), dtype=np.float32)
        edges.append(np.float32(e))
    edges.append(np.float32(np.inf))
    return np.array(edges, np.float32)


def owners(x, edges) -> np.ndarray:
    """Owning rank of each particle: slab r holds edges[r] <= x < edges[r+1]
    (the device-side test of k_mig_pack, in float32)."""
    xf = np.asarray(x, np.float32)
    return np.searchsorted(np.asarray(edges, np.float32)[1:-1], xf, side="right").astype(np.int32)


def ghost_capacity(x, edges, halo: float, factor: float = 3.0, floor: int = 4096) -> int:
    """Ghost / migrant slots per side: `factor` times the most particles
    within `halo` of any inner edge at the start (room for compression), plus
    `floor`."""
    xf = np.asarray(x, np.float32)
    worst = 0
    for e in np.asarray(edges, np.float32)[1:-1]:
        worst = max(worst, int(((xf >= e - halo) & (xf < e)).sum()), int(((xf >= e) & (xf < e + halo)).sum()))
    return int(factor * worst) + floor


DRIFT_ALLOWANCE = 1.5     # metres an owned particle may travel outside its slab in one tick


def default_halo(cfg, edges=None) -> float:
    """Ghost width D = 2h + DRIFT_ALLOWANCE (1.6 m at the default h = 0.05).
    2h so that every ghost the forces pass reads has all its own neighbours
    (no second exchange of ghost densities); the allowance is how far an
    owned particle may move outside its slab before the once-per-tick
    migration: 1.5 m, 180 m/s at dt = 1/120 s.  Measured on the metric scenes
    over 350 ticks (profiles/r01/slab_drift.json): at most 0.69 m per tick
    (MW2) and 0.62 m (M), speeds up to ~94 m/s (fluid struck by the
    pentagons).  Beyond the allowance the step fails loudly (ST_HALO_DRIFT).

    A slab between two neighbours must be at least 2D - 2h wide (the ghosts a
    rank needs come from its neighbours only); with `edges` the halo shrinks
    to fit the narrowest such slab (the small test scenes)."""
    h = float(cfg.gridConfig.smoothingLength)
    D = 2.0 * h + DRIFT_ALLOWANCE
    if edges is not None:
        w = np.diff(np.asarray(edges, np.float64))[1:-1]
        if len(w):
            D = min(D, (float(w.min()) + 2.0 * h) / 2.0)
    if not D > 2.0 * h:
        raise ValueError("slab decomposition: a slab is narrower than the 2h the halo needs")
    return D


def setup_rank(ctx, rank: int, nranks: int, fluid: dict, edges, cfg, rigids=None, halo=None,
               ghost_cap=None, domain=None):
    """Configure ctx as slab `rank` and upload the particles it owns (global
    ids = indices into `fluid`).  Returns the owned global ids."""
    import lpe  # the in-tree binding (little-physics-engine_amd/lpe.py)
    halo = default_halo(cfg, edges) if halo is None else halo
    w = np.diff(np.asarray(edges, np.float64))[1:-1]
    if len(w) and 2.0 * halo - 2.0 * float(cfg.gridConfig.smoothingLength) > float(w.min()):
        raise ValueError("slab decomposition: an inner slab is narrower than 2 * halo - 2h")
    x = np.asarray(fluid["x"], np.float32)
    if ghost_cap is None:
        ghost_cap = ghost_capacity(x, edges, halo)
    own = np.nonzero(owners(x, edges) == rank)[0].astype(np.int32)
    x0, x1 = float(edges[rank]), float(edges[rank + 1])
    ctx.sph_set_config(cfg)
    ctx.sph_set_slab(x0 if np.isfinite(x0) else 0.0, x1 if np.isfinite(x1) else 0.0, halo,
                     rank > 0, rank < nranks - 1, ghost_cap)
    sub = {k: np.asarray(fluid[k])[own] for k in ("x", "y", "vx", "vy", "mass", "density", "pressure")}
    ctx.sph_upload(sub["x"], sub["y"], sub["vx"], sub["vy"], sub["mass"], sub["density"], sub["pressure"])
    ctx.sph_set_ids(own)
    if domain is None:
        y = np.asarray(fluid["y"], np.float32)
        pad = 1.0
        domain = (float(x.min()) - pad, float(y.min()) - pad, float(x.max()) + pad, float(y.max()) + pad)
    ctx.sph_set_domain(*domain)
    ctx.sph_upload_rigids(rigids if rigids is not None else np.zeros(0, lpe.RIGID_DTYPE))
    return own


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
