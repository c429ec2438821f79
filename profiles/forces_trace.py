"""Round 4: per-block phase times of k_forces_couple (LDS-image version) on
the settled scene-M state, and the share of blocks whose neighbourhood did
not fit the image (sph_stats forcesGlobal).

    python3 profiles/snapshot.py --save 3000   (writes /tmp/lpe_snap.npz)
    LPE_LIB=profiles/_var/liblpe_ft.so python3 profiles/forces_trace.py

The library must be built with -DLPE_FTRACE (profiles/trace_build.sh sph ft -DLPE_FTRACE).
Stamps (lpe_sph.hip, FTR / FTRMAX): 0 block start, 1 after the image and the
pair list (barrier), 5 last wave out of the fluid loop, 2 pairs' geometry
done, 4 coupling done, 3 end; 6 lane-0 list length (max over waves), 7 the
image's record count (>= 100000: the block gathered from global memory)."""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe
z = np.load("/tmp/lpe_snap.npz")
ctx = lpe.Context(0)
ctx.rigid_set_config(lpe.rigid_config(universe=32.0))
ctx.sph_set_config(lpe.default_fluid_config())
ctx.rigid_upload(z["bodies"], z["verts"])
ctx.sph_upload(z["x"], z["y"], z["vx"], z["vy"], z["mass"], z["density"], z["pressure"])
ctx.world_set_coupling(None)
ctx.world_tick(1 / 120, 3); ctx.sync()
st0 = ctx.sph_stats()
L = lpe.lib()
ftr = hasattr(L, "lpe_ftrace")
nb = (len(z["x"]) + 255) // 256
if ftr:
    L.lpe_ftrace.argtypes = [C.c_int, C.c_void_p, C.c_int]
    buf = np.zeros(4096 * 8, np.uint64)
    L.lpe_ftrace(1, None, 0)
ctx.world_tick(1 / 120, 1); ctx.sync()
st1 = ctx.sph_stats()
print("forcesGlobal blocks per sub-step", (st1["forcesGlobal"] - st0["forcesGlobal"]) / 10.0, "of", nb,
      "stageFallback", st1["stageFallback"] - st0["stageFallback"])
if not ftr:
    sys.exit(0)
L.lpe_ftrace(0, buf.ctypes.data, buf.size)
W = 1024        # slots past the tiles' own: the filed blocks (QUARTER_BLOCKS, HALF_BLOCKS, COUPLED_MAX)
REG = (("quarter part blocks", 0, 512), ("half part blocks", 512, 832), ("coupled whole blocks", 832, 992))
pairs = None
if hasattr(L, "lpe_ftrace2"):
    L.lpe_ftrace2.argtypes = [C.c_void_p, C.c_int]
    buf2 = np.zeros(4096 * 8, np.uint64)
    L.lpe_ftrace2(buf2.ctypes.data, buf2.size)
    pairs = buf2[: (nb + W) * 8].reshape(nb + W, 8).astype(np.int64)
# slots: the tiles' blocks, then (round 5) the filed blocks by class; blocks
# that did not run a tile leave zeros
t = buf[: (nb + W) * 8].reshape(nb + W, 8).astype(np.int64)
ran = t[:, 0] > 0
region = np.full(len(ran), -1)
for r, (name, a, b) in enumerate(REG):
    region[nb + a: nb + b] = r
    print(name, int(ran[nb + a: nb + b].sum()))
isq = (region >= 0)[ran]
region = region[ran]
t = t[ran]
if pairs is not None:
    npairs_blk = pairs[ran][:, 5].copy()
    pairs = pairs[ran] / 100.0      # us since the pair's start, max over the block's lanes
nb = len(t)
t0 = t[:, 0].min()
us = lambda a, b: (t[:, b] - t[:, a]) / 100.0
start = (t[:, 0] - t0) / 100.0
end = (t[:, 3] - t0) / 100.0
has2 = t[:, 2] > 0
img = t[:, 7] < 100000
has6 = t[:, 6] > 0
cin = np.where(has6, us(5, 6), 0.0)
prs = np.where(has6 & has2, us(6, 2), 0.0)
fold = np.where(has2, us(2, 4), 0.0)
rows = [("start", start), ("stage+cand", us(0, 1)), ("fluid loop", us(1, 5)), ("coupling", us(5, 4)),
        ("  couple_in", cin), ("  pairs", prs), ("  fold+fin", fold),
        ("kick+write", us(4, 3)), ("end", end), ("img L", np.where(img, t[:, 7], t[:, 7] - 100000))]
print("kernel span us", end.max(), "blocks", nb, "image blocks", int(img.sum()))
print("pctl        " + " ".join(f"{p:>8}" for p in ("0", "50", "90", "99", "100")))
for name, v in rows:
    q = np.percentile(v, [0, 50, 90, 99, 100])
    print(f"{name:11s}", " ".join(f"{x:8.1f}" for x in q))
for name, sel in [("tile blocks", ~isq)] + [(REG[r][0], region == r) for r in range(len(REG))]:
    if sel.any():
        print(f"{name:20s} n {int(sel.sum()):5d}  start pctl 0/50/90/100:",
              " ".join(f"{x:6.1f}" for x in np.percentile(start[sel], [0, 50, 90, 100])),
              " end:", " ".join(f"{x:6.1f}" for x in np.percentile(end[sel], [0, 50, 90, 100])))
print("slowest blocks: blk img L stage fluid couple (in pairs fold) kick end")
for k in np.argsort(-end)[:10]:
    print(("q" if isq[k] else "") + str(k), int(img[k]), t[k, 7] % 100000, round(us(0, 1)[k], 1), round(us(1, 5)[k], 1), round(us(5, 4)[k], 1),
          "(", round(cin[k], 1), round(prs[k], 1), round(fold[k], 1), ")", round(us(4, 3)[k], 1), round(end[k], 1),
          "" if pairs is None else "pair stages (record, pip, closest, impulse+atomics): %s" %
          [round(float(x), 2) for x in pairs[k, :4]], "pairs", int(npairs_blk[k]))
if pairs is not None:
    has = npairs_blk > 0
    print("blocks with coupling pairs", int(has.sum()), "pairs per block pctl 50/90/99/100:",
          np.percentile(npairs_blk[has], [50, 90, 99, 100]).round(0).tolist() if has.any() else None)
