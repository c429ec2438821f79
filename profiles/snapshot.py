"""Settle scene M and save its state (--save PREP), or run K ticks from the saved state (--load K):
the settled state without paying the 3000 settling ticks in every profiling run.
FIRST=1: time the first tick after re-uploading the state (physics-identical across library variants)."""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe, scenes
path = "/tmp/lpe_snap.npz"
s = scenes.scene("M"); fl = s["fluid"]; b, v = scenes.to_bodies(s["bodies"])
ctx = lpe.Context(0)
ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
ctx.sph_set_config(lpe.default_fluid_config())
if sys.argv[1] == "--save":
    ctx.rigid_upload(b, v)
    ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
    ctx.world_set_coupling(None)
    ctx.world_tick(1 / 120, int(sys.argv[2])); ctx.sync()
    d = ctx.sph_download(); bb = ctx.rigid_download()
    np.savez(path, bodies=bb, verts=v, mass=fl["mass"], **{k: d[k] for k in ("x", "y", "vx", "vy", "density", "pressure")})
    print("saved", len(d["x"]), len(bb))
else:
    z = np.load(path)
    ctx.rigid_upload(z["bodies"], z["verts"])
    ctx.sph_upload(z["x"], z["y"], z["vx"], z["vy"], z["mass"], z["density"], z["pressure"])
    ctx.world_set_coupling(None)
    k = int(sys.argv[2])
    ctx.world_tick(1 / 120, 3); ctx.sync()
    t0 = time.perf_counter(); ctx.world_tick(1 / 120, k); ctx.sync()
    r = k / (time.perf_counter() - t0)
    ctx.timing(1); ctx.timing_reset(); ctx.world_tick(1 / 120, 10); t = ctx.timing_read(); ctx.timing(0)
    ks = {kk: round(vv[0] / max(vv[1], 1) * 1e3, 2) for kk, vv in t.items()}
    top = dict(sorted(ks.items(), key=lambda kv: -kv[1])[:int(os.environ.get("TOPK", "8"))])
    print(os.environ.get("LPE_LIB", "default"), "ticks/s", round(r, 1), top)
    if os.environ.get("FIRST"):
        ctx.rigid_upload(z["bodies"], z["verts"])
        ctx.sph_upload(z["x"], z["y"], z["vx"], z["vy"], z["mass"], z["density"], z["pressure"])
        ctx.timing(1); ctx.timing_reset(); ctx.world_tick(1 / 120, 1); t = ctx.timing_read(); ctx.timing(0)
        print("  first tick:", {kk: round(vv[0] / max(vv[1], 1) * 1e3, 2) for kk, vv in t.items() if kk in ("k_forces_couple", "k_density")})
    if os.environ.get("DIAG"):
        ctx.sph_diag(True); ctx.world_tick(1 / 120, 1); st = ctx.sph_stats(); ctx.sph_diag(False)
        print({k: st[k] for k in ("rigidCandidates", "neighbours", "maxCellOccupancy", "nlistOverflow")}, "per particle-substep cand", st["rigidCandidates"] / (10 * len(z["x"])))
ctx.close()
