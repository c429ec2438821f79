"""Diagnostic (round 6): the capped-cell slab failure at M@240 -- cell counts near the edges."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe, scenes  # noqa
import test_slab_gpu as T  # noqa
s, fl, bodies, verts = T._m_state(240)
cfg = lpe.default_fluid_config()
cs = T.slab.cell_size(cfg)
eps = np.float32(cfg.gridConfig.gridEpsilon)
col = np.floor((fl["x"] + eps) / np.float32(cs)).astype(np.int64)
row = np.floor((fl["y"] + eps) / np.float32(cs)).astype(np.int64)
cells, counts = np.unique(np.stack([col, row], 1), axis=0, return_counts=True)
print("max count", counts.max(), "cells over 64:", (counts > 64).sum(), "over 129:", (counts > 129).sum())
over = np.unique(cells[counts > 64][:, 0])
print("over-full columns", over.tolist())
print("global col range", col.min(), col.max())
for nr in (2,):
    pick = over[np.linspace(0, len(over) - 1, nr + 1).astype(int)[1:-1]]
    cuts = sorted(set(int(c) + d for c, d in zip(pick, (1, 0, -1))))
    print("cuts", cuts)
    for c in cuts:
        for dc in range(-4, 5):
            sel = cells[:, 0] == c + dc
            print("  col", c + dc, "max", counts[sel].max() if sel.any() else 0)
# per tick: single domain capped, max counts near the cut; the 2-rank run tick by tick
cut = cuts[0]
one = lpe.Context(0)
one.rigid_set_config(lpe.rigid_config(universe=s["U"])); one.rigid_upload(bodies, verts)
one.sph_set_config(cfg)
one.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
one.world_set_coupling(np.arange(len(bodies) - 1, -1, -1, dtype=np.int32))
one.sph_set_mode(lpe.SPH_MODE_REF_CELL_CAP)
for t in range(3):
    one.world_tick(T.DT, 1)
    o = one.sph_download()
    c2 = np.floor((o["x"] + eps) / np.float32(cs)).astype(np.int64)
    r2 = np.floor((o["y"] + eps) / np.float32(cs)).astype(np.int64)
    cl, ct = np.unique(np.stack([c2, r2], 1), axis=0, return_counts=True)
    print("tick", t + 1, "max", ct.max(), {int(c): int(ct[cl[:, 0] == c].max()) for c in range(cut - 4, cut + 4) if (cl[:, 0] == c).any()})
one.close()
edges = np.array([-np.inf, cut * cs, np.inf], np.float32)
ctxs = [lpe.Context(0) for _ in range(2)]
for r, c in enumerate(ctxs):
    c.rigid_set_config(lpe.rigid_config(universe=s["U"])); c.rigid_upload(bodies, verts)
    T.slab.setup_rank(c, r, 2, fl, edges, cfg, cells="ref")
    c.world_set_coupling(np.arange(len(bodies) - 1, -1, -1, dtype=np.int32))
    print("rank", r, c.sph_slab_info())
for t in range(3):
    try:
        lpe.mg_loopback_run(ctxs, 1, world=lpe.WorldConfig(T.DT, 1.0, 1.0, 1.0))
        for c in ctxs:
            c.sph_download_owned(cap=len(fl["x"]))
        print("slab tick", t + 1, "ok")
    except lpe.LpeError as e:
        print("slab tick", t + 1, e)
        break
