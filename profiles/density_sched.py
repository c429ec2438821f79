"""Round 6: where the tick's density pass (k_density<true>) put its tiles
(XCC / SE / CU from HW_ID, DTRHW) and how long each took, on the settled
scene-M state: is the pass's span one slow tile, or a CU holding several?

    python3 profiles/snapshot.py --save 3000   (writes /tmp/lpe_snap.npz)
    LPE_LIB=profiles/_var/liblpe_NAME.so python3 profiles/density_sched.py [OUT.npz]

Library built with -DLPE_FTRACE -DLPE_FTRACE_LITE -DLPE_FTRACE_NOCPT.  The
prelaunch is switched off (LPE_NO_PRELAUNCH) so that the stamps are the
tick's last sub-step's pass on the context stream."""
import ctypes as C, os, sys
import numpy as np
os.environ["LPE_NO_PRELAUNCH"] = "1"
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
L.lpe_dtrace.argtypes = [C.c_void_p, C.c_int]
nb = (len(z["x"]) + 255) // 256
runs = []
for rep in range(int(os.environ.get("REPS", "3"))):
    L.lpe_ftrace(1, None, 0)
    ctx.world_tick(1 / 120, 1); ctx.sync()
    buf = np.zeros(4096 * 8, np.uint64)
    L.lpe_dtrace(buf.ctypes.data, buf.size)
    L.lpe_ftrace(0, None, 0)
    runs.append(buf[: nb * 8].reshape(nb, 8).astype(np.int64))
if len(sys.argv) > 1:
    np.savez(sys.argv[1], t=np.stack(runs), nb=nb)
for rep, t in enumerate(runs):
    ran = t[:, 0] > 0
    idx = np.where(ran)[0]
    t = t[ran]
    t0 = t[:, 0].min()
    st = (t[:, 0] - t0) / 100.0
    en = (t[:, 4] - t0) / 100.0
    walk = (t[:, 2] - t[:, 1]) / 100.0
    stage = (t[:, 1] - t[:, 0]) / 100.0
    d = en - st
    hw = t[:, 7]
    xcc = (hw >> 24) & 0xF
    key = xcc * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 16 + ((hw >> 8) & 15)
    ucu = np.unique(key)
    fin = np.array([en[key == k].max() for k in ucu])
    tot = np.array([d[key == k].sum() for k in ucu])
    n = np.array([(key == k).sum() for k in ucu])
    print(f"--- pass {rep}: span {en.max():.1f} us, {len(t)} tiles on {len(ucu)} CUs, tile-us {d.sum():.0f} "
          f"(/1024 slots {d.sum() / 1024:.1f})")
    print("  start pctl 50/90/100", np.percentile(st, [50, 90, 100]).round(1),
          " tile dur 10/50/90/100", np.percentile(d, [10, 50, 90, 100]).round(1),
          " stage 50/90", np.percentile(stage, [50, 90]).round(1), " walk 50/90/100", np.percentile(walk, [50, 90, 100]).round(1))
    print("  tiles per CU", np.bincount(n).tolist(), " CU finish 0/50/90/100", np.percentile(fin, [0, 50, 90, 100]).round(1),
          " CU tile-us 0/50/90/100", np.percentile(tot, [0, 50, 90, 100]).round(1))
    # the slowest tiles and their CU mates
    for i in np.argsort(-en)[:5]:
        mates = np.where(key == key[i])[0]
        print(f"  tile {idx[i]} dur {d[i]:.1f} (stage {stage[i]:.1f} walk {walk[i]:.1f} longest list {t[i, 5]}) CU {key[i]}: mates",
              [(int(idx[m]), round(float(d[m]), 1)) for m in mates if m != i])
    # tile index vs CU: how are consecutive tiles spread
    order = np.argsort(idx)
    print("  first 16 tiles' CUs:", key[order[:16]].tolist())
    # duration along the tile index (spatial) in 32 bins
    binned = [round(float(d[order][k:k + 32].mean()), 1) for k in range(0, len(order), 32)]
    print("  mean tile dur per 32 tiles:", binned)
