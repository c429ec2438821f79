"""Round 6: where k_forces_couple's blocks ran (XCC, SE, CU from the block's
HW_ID / XCC_ID) and when, on the settled scene-M state — how well the launch
packs its blocks onto the 1,024 resident slots (4 per CU).

    python3 profiles/snapshot.py --save 3000   (writes /tmp/lpe_snap.npz)
    LPE_LIB=profiles/_var/liblpe_ft.so python3 profiles/forces_sched.py [OUT.npz]

Library built with -DLPE_FTRACE (profiles/trace_build.sh sph ft -DLPE_FTRACE).
Stamps as in forces_trace.py; ftrace2 slot 5 the block's coupling pairs,
slots 6 / 7 the block's HW_ID / XCC_ID (FTRHW)."""
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
L = lpe.lib()
L.lpe_ftrace.argtypes = [C.c_int, C.c_void_p, C.c_int]
L.lpe_ftrace2.argtypes = [C.c_void_p, C.c_int]
nb = (len(z["x"]) + 255) // 256
W = 1024
REG = (("quarter", 0, 512), ("half", 512, 832), ("coupled", 832, 992))
runs = []
for rep in range(int(os.environ.get("REPS", "3"))):
    buf = np.zeros(4096 * 8, np.uint64)
    buf2 = np.zeros(4096 * 8, np.uint64)
    L.lpe_ftrace(1, None, 0)
    ctx.world_tick(1 / 120, 1); ctx.sync()
    L.lpe_ftrace(0, buf.ctypes.data, buf.size)
    L.lpe_ftrace2(buf2.ctypes.data, buf2.size)
    runs.append((buf[: (nb + W) * 8].reshape(nb + W, 8).astype(np.int64),
                 buf2[: (nb + W) * 8].reshape(nb + W, 8).astype(np.int64)))
if len(sys.argv) > 1:
    np.savez(sys.argv[1], t=np.stack([r[0] for r in runs]), t2=np.stack([r[1] for r in runs]), nb=nb)

for rep, (t, t2) in enumerate(runs):
    kind = np.full(nb + W, "tile", dtype=object)
    for name, a, b in REG:
        kind[nb + a: nb + b] = name
    # the last launch's blocks: start within 200 us of the latest start
    ran = (t[:, 0] > 0) & (t[:, 3] > 0)
    tmax = t[ran, 0].max()
    ran &= t[:, 0] > tmax - 20000
    t, t2, kind = t[ran], t2[ran], kind[ran]
    t0 = t[:, 0].min()
    st = (t[:, 0] - t0) / 100.0
    en = (t[:, 3] - t0) / 100.0
    dur = en - st
    hw = t2[:, 6]
    xcc = t2[:, 7] & 0xF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 0x7
    key = xcc * 1000 + se * 100 + sh * 16 + cu
    ucu = np.unique(key)
    print(f"--- launch {rep}: span {en.max():.1f} us, {len(t)} blocks on {len(ucu)} CUs "
          f"({len(np.unique(xcc))} XCCs), block-us total {dur.sum():.0f} -> /1024 slots {dur.sum() / 1024:.1f} us")
    for k in ("quarter", "half", "coupled", "tile"):
        sel = kind == k
        if sel.any():
            print(f"  {k:8s} n {sel.sum():4d} dur pctl 10/50/90/100 "
                  + " ".join(f"{x:5.1f}" for x in np.percentile(dur[sel], [10, 50, 90, 100]))
                  + "  start 50/90/100 " + " ".join(f"{x:5.1f}" for x in np.percentile(st[sel], [50, 90, 100])))
    fin = np.array([en[key == k].max() for k in ucu])
    busy = np.array([dur[key == k].sum() for k in ucu])
    nblk = np.array([(key == k).sum() for k in ucu])
    print("  CU finish pctl 0/10/50/90/100", " ".join(f"{x:5.1f}" for x in np.percentile(fin, [0, 10, 50, 90, 100])))
    print("  CU busy (block-us) pctl 0/10/50/90/100", " ".join(f"{x:5.1f}" for x in np.percentile(busy, [0, 10, 50, 90, 100])))
    print("  blocks per CU pctl 0/50/100", np.percentile(nblk, [0, 50, 100]).tolist())
    xf = {int(x): float(en[xcc == x].max()) for x in np.unique(xcc)}
    xb = {int(x): float(dur[xcc == x].sum()) for x in np.unique(xcc)}
    print("  per XCC finish", {k: round(v, 1) for k, v in xf.items()})
    print("  per XCC block-us", {k: round(v) for k, v in xb.items()})
    # the latest CUs' block sequences
    for k in ucu[np.argsort(-fin)[:4]]:
        sel = np.where(key == k)[0]
        sel = sel[np.argsort(st[sel])]
        print(f"  CU {k}: " + "; ".join(f"{kind[i][0]}{st[i]:.1f}-{en[i]:.1f}({t2[i, 5]}p)" for i in sel))
    # concurrency over time
    grid = np.arange(0, en.max() + 1, 2.0)
    conc = [(np.sum((st <= g) & (en > g))) for g in grid]
    print("  resident blocks every 2 us:", conc)
