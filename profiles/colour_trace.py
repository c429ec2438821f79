"""Per-group stage times of k_group_colour (round 4): the list compaction
over all candidate pairs, the barrier, and wave 0's colouring chain; and the
stages of k_stripe_setup before it.

    profiles/trace_build.sh rigid pt -DLPE_PTRACE
    LPE_LIB=profiles/_var/liblpe_pt.so python3 profiles/colour_trace.py

Runs the rigid microbench fixture (tests/golden/pile_M_t250.npz) and the C1 /
C3 scenes after their settle, and prints per group: candidate pairs (np),
listed pairs, stripe slots, colours, and the µs of each stage (wall_clock64,
100 MHz)."""
import ctypes as C
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import lpe  # noqa: E402

spec = importlib.util.spec_from_file_location("scenes", os.path.join(ROOT, "little-physics-engine_amd", "scenes.py"))
scenes = importlib.util.module_from_spec(spec)
spec.loader.exec_module(scenes)
L = lpe.lib()
L.lpe_ctrace.argtypes = [C.c_void_p]
DT = 1.0 / 120.0


def report(name):
    buf = np.zeros(129 * 8, np.uint64)
    L.lpe_ctrace(buf.ctypes.data)
    t = buf.reshape(129, 8).astype(np.int64)
    st = t[128]
    print(f"{name}: k_stripe_setup stages (us): stripe count {(st[1] - st[0]) / 100:.2f}, pair pass "
          f"{(st[2] - st[1]) / 100:.2f}, bodies {(st[3] - st[2]) / 100:.2f}, prefixes {(st[4] - st[3]) / 100:.2f}, "
          f"body slots {(st[5] - st[4]) / 100:.2f}; total {(st[5] - st[0]) / 100:.2f}")
    last = t[:, 0].max()
    rows = [g for g in range(128) if t[g, 0] > 0 and last - t[g, 0] < 100000 and t[g, 3] >= t[g, 0]]
    t0 = min(t[g, 0] for g in rows)
    print(f"{name}: {len(rows)} groups; kernel span {(max(t[g, 3] for g in rows) - t0) / 100:.2f} us")
    for g in rows[:12]:
        r = t[g]
        print(f"  g{g:3d} np {r[4]:6d} pairs {r[5]:5d} slots {r[6]:5d} colours {r[7]:2d}  "
              f"entry +{(r[0] - t0) / 100:6.2f}  list {(r[1] - r[0]) / 100:6.2f}  barrier {(r[2] - r[1]) / 100:5.2f}"
              f"  chain {(r[3] - r[2]) / 100:6.2f} us ({(r[3] - r[2]) / 100 / max(r[5], 1) * 1000:.0f} ns a pair)")


z = np.load(os.path.join(ROOT, "tests", "golden", "pile_M_t250.npz"))
ctx = lpe.Context(0)
ctx.rigid_set_config(lpe.rigid_config(universe=32.0))
for _ in range(3):
    ctx.rigid_upload(z["bodies"], z["verts"])
    ctx.rigid_step()
ctx.sync()
report("pile_M fixture")
ctx.close()
for sc, prep in (("C1", 60), ("C3", 240)):
    s = scenes.rigid_scene(sc)
    b, v = scenes.to_bodies(s["bodies"])
    c = lpe.Context(0)
    c.rigid_set_config(lpe.rigid_config(universe=s["U"], pgs_iterations=s["pgs_iterations"]))
    c.rigid_upload(b, v)
    c.world_tick(DT, prep)
    c.sync()
    report(sc)
    c.close()
