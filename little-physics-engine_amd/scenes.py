"""Seeded synthetic scenes and the reference's gathers.

The reference scenarios seed from time() (simple_fluid.cpp:130,
fluid_and_polygons.cpp:126), so scenes here come from this generator
(numpy PCG64 with a fixed seed) and reuse the reference's entity recipes:
walls after makeWall / makeBoundaryWall (simple_fluid.cpp:19-54), pentagons
after fluid_and_polygons.cpp:141-160, fluid lattices after
simple_fluid.cpp:131-139.  Creation order is walls, then rigids, then fluid.
"""
from __future__ import annotations

import math

import numpy as np

try:
    from . import lpe as _lpe  # type: ignore
except ImportError:  # loaded by path
    import importlib.util
    import os
    _spec = importlib.util.spec_from_file_location(
        "lpe", os.path.join(os.path.dirname(os.path.abspath(__file__)), "lpe.py"))
    _lpe = importlib.util.module_from_spec(_spec)
    _spec.loader.exec_module(_lpe)

RIGID_DTYPE = _lpe.RIGID_DTYPE
MAX_POLY_VERTS = _lpe.MAX_POLY_VERTS

LATTICE_S = 0.025                    # lattice spacing s = h/2
FLUID_MASS = 0.5 * LATTICE_S ** 2    # m = rho0 * s^2 (rho0 = 0.5, fluid.hpp:135)
WALL_MASS = 1e30
WALL_THICK = 0.1


# ---------------------------------------------------------------------------
# shape builders (polygon.hpp:154-284), double precision
def regular_polygon(sides: int, sz: float) -> np.ndarray:
    """buildRegularPolygon (polygon.hpp:154-167): (sz cos a, -sz sin a)."""
    step = 2.0 * math.pi / float(sides)
    return np.array([(sz * math.cos(i * step), -sz * math.sin(i * step)) for i in range(sides)],
                    dtype=np.float64)


def random_convex_polygon(rng, sz: float) -> np.ndarray:
    """buildRandomConvexPolygon (polygon.hpp:182-203) with this generator's rng."""
    sides = int(rng.integers(3, 8))
    step = 2.0 * math.pi / float(sides)
    angle = 0.0
    out = []
    for _ in range(sides):
        r = float(rng.uniform(0.5 * sz, sz))
        out.append((r * math.cos(angle), -r * math.sin(angle)))
        angle += step
    return np.array(out, dtype=np.float64)


def polygon_inertia(verts: np.ndarray, mass: float) -> float:
    """calculatePolygonInertia (polygon.hpp:266-284), same summation order."""
    num = 0.0
    den = 0.0
    n = len(verts)
    for i in range(n):
        j = (i + 1) % n
        xi, yi = float(verts[i, 0]), float(verts[i, 1])
        xj, yj = float(verts[j, 0]), float(verts[j, 1])
        cross = xi * yj - yi * xj
        num += cross * ((xi * xi + yi * yi) + (xi * xj + yi * yj) + (xj * xj + yj * yj))
        den += cross
    return (mass * num) / (6.0 * den)


# ---------------------------------------------------------------------------
class Bodies:
    """Solid bodies in creation order (walls first).  Mirrors the components
    the reference's rigid path reads: Position, Velocity, Mass, AngularPosition,
    AngularVelocity, Inertia, Boundary, Sleep, PolygonShape / CircleShape."""

    def __init__(self):
        self.rows = []

    def add(self, **kw):
        row = dict(x=0.0, y=0.0, vx=0.0, vy=0.0, mass=1.0, angle=0.0, omega=0.0,
                   has_angpos=True, has_angvel=False, has_inertia=False, inertia=1.0,
                   boundary=False, has_sleep=True, asleep=False, sleep_counter=0,
                   circle=False, radius=0.0, verts=None, shape_size=0.0)
        row.update(kw)
        self.rows.append(row)

    def __len__(self):
        return len(self.rows)


def add_walls(b: Bodies, U: float):
    """Four Boundary walls (simple_fluid.cpp:19-54, :87-108): mass 1e30, asleep."""
    hw = WALL_THICK * 0.5
    for (cx, cy, halfW, halfH) in ((0.0, U * 0.5, hw, U * 0.5), (U, U * 0.5, hw, U * 0.5),
                                   (U * 0.5, 0.0, U * 0.5, hw), (U * 0.5, U, U * 0.5, hw)):
        verts = np.array([(-halfW, -halfH), (-halfW, halfH), (halfW, halfH), (halfW, -halfH)],
                         np.float64)
        b.add(x=cx, y=cy, mass=WALL_MASS, boundary=True, asleep=True, sleep_counter=9999999,
              verts=verts, shape_size=halfH, has_angvel=False, has_inertia=False)


def add_pentagon_lattice(b: Bodies, rng, nx, ny, x0, y0, pitch, radius_fn, mass_mean=5.0,
                         mass_std=0.2, vel_scale=0.5):
    """Pentagons after fluid_and_polygons.cpp:141-160 on an nx x ny lattice."""
    i = 0
    for row in range(ny):
        for col in range(nx):
            r = radius_fn(i)
            verts = regular_polygon(5, r)
            mass = max(0.1, float(rng.normal(mass_mean, mass_std)))
            vx = float(rng.normal(0.0, vel_scale)) * 0.2
            vy = abs(float(rng.normal(0.0, vel_scale)))
            b.add(x=x0 + col * pitch, y=y0 + row * pitch, vx=vx, vy=vy, mass=mass,
                  verts=verts, shape_size=r, has_angvel=True, has_inertia=True,
                  inertia=polygon_inertia(verts, mass))
            i += 1


def fluid_lattice(rng, nx, ny, x0, y0, s=LATTICE_S, mass=FLUID_MASS):
    """nx x ny lattice at spacing s with uniform jitter +-0.1 s
    (simple_fluid.cpp:131-139).  Row-major creation order; float64 like the ECS."""
    col = np.tile(np.arange(nx, dtype=np.float64), ny)
    row = np.repeat(np.arange(ny, dtype=np.float64), nx)
    jx = rng.uniform(-0.1, 0.1, nx * ny) * s
    jy = rng.uniform(-0.1, 0.1, nx * ny) * s
    x = x0 + (col + 0.5) * s + jx
    y = y0 + (row + 0.5) * s + jy
    n = nx * ny
    return dict(x=x, y=y, vx=np.zeros(n), vy=np.zeros(n), mass=np.full(n, mass),
                density=np.zeros(n), pressure=np.zeros(n))


# ---------------------------------------------------------------------------
def gather_rigids(b: Bodies, order=None) -> np.ndarray:
    """FluidSystem::gatherRigidBodies (fluid.cpp:304-438) for the given body
    order: float pose, polygon world verts computed in double from
    cos/sin of float(angle) in float precision (the reference calls
    std::cos(float), fluid.cpp:399-400) and cast to float, AABB of the float
    verts; circles use
    float radius.  Missing mass/inertia default to 1."""
    idx = list(range(len(b))) if order is None else list(order)
    out = np.zeros(len(idx), RIGID_DTYPE)
    for k, i in enumerate(idx):
        r = b.rows[i]
        rb = out[k]
        posX = np.float32(r["x"])
        posY = np.float32(r["y"])
        angle = np.float32(r["angle"]) if r["has_angpos"] else np.float32(0.0)
        rb["posX"], rb["posY"], rb["angle"] = posX, posY, angle
        rb["vx"], rb["vy"] = np.float32(r["vx"]), np.float32(r["vy"])
        rb["omega"] = np.float32(r["omega"]) if r["has_angvel"] else np.float32(0.0)
        rb["mass"] = np.float32(r["mass"])
        rb["inertia"] = np.float32(r["inertia"]) if r["has_inertia"] else np.float32(1.0)
        if r["circle"]:
            rad = np.float32(r["radius"])
            rb["shapeType"] = 0
            rb["radius"] = rad
            rb["vertCount"] = 0
            rb["minX"], rb["maxX"] = posX - rad, posX + rad
            rb["minY"], rb["maxY"] = posY - rad, posY + rad
        else:
            verts = r["verts"][:MAX_POLY_VERTS]
            rb["shapeType"] = 1
            rb["vertCount"] = len(verts)
            c = float(np.float32(math.cos(float(angle))))
            s = float(np.float32(math.sin(float(angle))))
            wx = np.array([r["x"] + (lx * c - ly * s) for lx, ly in verts], np.float64)
            wy = np.array([r["y"] + (lx * s + ly * c) for lx, ly in verts], np.float64)
            fx = wx.astype(np.float32)
            fy = wy.astype(np.float32)
            rb["vertsX"][:len(verts)] = fx
            rb["vertsY"][:len(verts)] = fy
            rb["minX"], rb["maxX"] = fx.min(), fx.max()
            rb["minY"], rb["maxY"] = fy.min(), fy.max()
    return out


# ---------------------------------------------------------------------------
# named scenes
def scene(name: str):
    """Returns dict(U, fluid, bodies, seed, desc)."""
    if name == "C2":     # 64k SPH dam break, U = 20 m, R = 4 walls
        U, seed = 20.0, 2
        rng = np.random.default_rng(seed)
        b = Bodies()
        add_walls(b, U)
        fl = fluid_lattice(rng, 256, 256, 0.15, U - 0.15 - 256 * LATTICE_S)
        return dict(U=U, fluid=fl, bodies=b, seed=seed, desc="C2: 256x256 dam break, U=20")
    if name == "C4":     # 256k SPH + 512 pentagons, U = 32 m
        U, seed = 32.0, 4
        rng = np.random.default_rng(seed)
        b = Bodies()
        add_walls(b, U)
        sizes = (0.25, 0.35, 0.45)
        fx0 = 0.5 * (U - 512 * LATTICE_S)
        add_pentagon_lattice(b, rng, 32, 16, 0.5 * (U - 31 * 0.9), U - 0.15 - 512 * LATTICE_S - 16 * 0.9,
                             0.9, lambda i: sizes[i % 3])
        fl = fluid_lattice(rng, 512, 512, fx0, U - 0.15 - 512 * LATTICE_S)
        return dict(U=U, fluid=fl, bodies=b, seed=seed, desc="C4: 512x512 SPH + 512 pentagons, U=32")
    if name == "M":      # metric scene: 256k SPH + 4096 pentagons (+4 walls), U = 32 m
        U, seed = 32.0, 6
        rng = np.random.default_rng(seed)
        b = Bodies()
        add_walls(b, U)
        pool_top = U - 0.15 - 256 * LATTICE_S
        add_pentagon_lattice(b, rng, 128, 32, 0.5 * (U - 127 * 0.24), pool_top - 0.3 - 31 * 0.24,
                             0.24, lambda i: 0.1)
        fl = fluid_lattice(rng, 1024, 256, 0.5 * (U - 1024 * LATTICE_S), pool_top)
        return dict(U=U, fluid=fl, bodies=b, seed=seed,
                    desc="M: 1024x256 SPH pool + 4096 pentagons (128x32 @0.24 m), U=32")
    if name == "C5":     # 2M SPH for the 8-GPU strong-scaling config: 2048 x 1024 lattice + 4 walls, U = 64 m
        U, seed = 64.0, 5
        rng = np.random.default_rng(seed)
        b = Bodies()
        add_walls(b, U)
        fl = fluid_lattice(rng, 2048, 1024, 0.5 * (U - 2048 * LATTICE_S), U - 0.15 - 1024 * LATTICE_S)
        return dict(U=U, fluid=fl, bodies=b, seed=seed,
                    desc="C5: 2048x1024 SPH (51.2 x 25.6 m) + 4 walls, U=64")
    if name.startswith("MW"):   # M widened N x for weak scaling: N x 256k SPH, the same 4096-pentagon pile
        nw = int(name[2:] or 1)
        U, seed = 32.0 * nw, 6
        rng = np.random.default_rng(seed)
        b = Bodies()
        add_walls(b, U)
        pool_top = U - 0.15 - 256 * LATTICE_S
        add_pentagon_lattice(b, rng, 128, 32, 0.5 * (U - 127 * 0.24), pool_top - 0.3 - 31 * 0.24,
                             0.24, lambda i: 0.1)
        fl = fluid_lattice(rng, 1024 * nw, 256, 0.5 * (U - 1024 * nw * LATTICE_S), pool_top)
        return dict(U=U, fluid=fl, bodies=b, seed=seed,
                    desc=f"MW{nw}: {1024 * nw}x256 SPH pool + the M pile of 4096 pentagons "
                         f"(128x32 @0.24 m, centred), U={U:g}")
    if name.startswith("small"):   # test scenes: small{N} fluid + a few rigids
        parts = name[5:].split("_")
        side = int(parts[0]) if parts and parts[0] else 64
        nrig = int(parts[1]) if len(parts) > 1 else 8
        U, seed = 6.0, 11 + side + nrig
        rng = np.random.default_rng(seed)
        b = Bodies()
        add_walls(b, U)
        x0 = 0.5 * (U - side * LATTICE_S)
        top = U - 0.15 - side * LATTICE_S
        if nrig:
            ncol = max(1, int(math.ceil(math.sqrt(nrig))))
            nrow = (nrig + ncol - 1) // ncol
            add_pentagon_lattice(b, rng, ncol, nrow, x0 + 0.2, top + 0.12, 0.3,
                                 lambda i: 0.1 + 0.02 * (i % 3))
            del b.rows[4 + nrig:]
        fl = fluid_lattice(rng, side, side, x0, top)
        return dict(U=U, fluid=fl, bodies=b, seed=seed, desc=f"small: {side}^2 fluid + {nrig} pentagons")
    raise KeyError(name)


def to_bodies(b: Bodies, eid_base: int = 1):
    """lpe_body array + shared local-vertex array, in creation order.  Entity
    ids follow a fresh registry: SimulatorState is entity 0 (sim.cpp:95-96),
    bodies are created next."""
    L = _lpe
    out = np.zeros(len(b), L.BODY_DTYPE)
    verts = []
    for i, r in enumerate(b.rows):
        f = L.BODY_HAS_PHASE | L.BODY_SOLID | L.BODY_HAS_MASS | L.BODY_HAS_VEL
        if r["boundary"]:
            f |= L.BODY_BOUNDARY
        if r["has_sleep"]:
            f |= L.BODY_HAS_SLEEP
        if r["asleep"]:
            f |= L.BODY_ASLEEP
        if r["has_angpos"]:
            f |= L.BODY_HAS_ANGPOS
        if r["has_angvel"]:
            f |= L.BODY_HAS_ANGVEL
        if r["has_inertia"]:
            f |= L.BODY_HAS_INERTIA
        o = out[i]
        o["eid"] = eid_base + i
        if r["circle"]:
            f |= L.BODY_CIRCLE
            o["radius"] = r["radius"]
            o["vert_off"] = len(verts) // 2
            o["vert_cnt"] = 0
        else:
            f |= L.BODY_POLYGON
            o["vert_off"] = len(verts) // 2
            o["vert_cnt"] = len(r["verts"])
            verts.extend(np.asarray(r["verts"], np.float64).ravel().tolist())
        o["flags"] = f
        for k in ("x", "y", "angle", "vx", "vy", "omega", "mass", "inertia"):
            o[k] = r[k]
        o["sleep_counter"] = r["sleep_counter"]
    return out, np.array(verts if verts else [0.0, 0.0], np.float64)


def rigid_scene(name: str):
    """Rigid-only scenes: returns dict(U, bodies, desc, pgs_iterations)."""
    if name == "C1":     # 128-box stack, U = 6 m, seed 1
        U = 6.0
        b = Bodies()
        add_walls(b, U)
        box = regular_polygon(4, 0.2)
        half = 0.2 * math.cos(math.pi / 4)
        floor = U - WALL_THICK * 0.5
        for row in range(16):
            for col in range(8):
                x = 0.5 * U + (col - 3.5) * 0.4
                y = floor - half - 0.002 - row * 0.29
                b.add(x=x, y=y, mass=1.0, angle=math.pi / 4, verts=box, shape_size=0.2,
                      has_angvel=True, has_inertia=True, inertia=polygon_inertia(box, 1.0))
        return dict(U=U, bodies=b, pgs_iterations=10, desc="C1: 8x16 box stack, U=6")
    if name.startswith("C3") or name.startswith("pile"):
        # C3: 64x64 random-polygon pile (random_polygons.cpp:133-207 recipe,
        # sizes 0.1-0.25), U = 40 m, 16 PGS iterations; pile{k}: k x k version
        k = 64 if name.startswith("C3") else int(name[4:])
        U = 40.0 if k >= 32 else max(6.0, 0.55 * k + 2.0)
        rng = np.random.default_rng(3 + (0 if k == 64 else 1000 + k))
        b = Bodies()
        add_walls(b, U)
        x0 = 0.5 * (U - (k - 1) * 0.55)
        y0 = U - 0.3 - (k - 1) * 0.55
        for row in range(k):
            for col in range(k):
                size = float(rng.uniform(0.1, 0.25))
                if rng.uniform() < 0.6:
                    verts = regular_polygon(int(rng.integers(3, 9)), size)
                else:
                    verts = random_convex_polygon(rng, size)
                mass = max(0.1, float(rng.normal(1.0, 0.1)))
                b.add(x=x0 + col * 0.55, y=y0 + row * 0.55, vx=float(rng.uniform(-2, 2)),
                      vy=float(rng.uniform(-2, 2)), mass=mass, omega=float(rng.uniform(-1, 1)),
                      verts=verts, shape_size=size, has_angvel=True, has_inertia=True,
                      inertia=polygon_inertia(verts, mass))
        return dict(U=U, bodies=b, pgs_iterations=16 if k == 64 else 10,
                    desc=f"{'C3' if k == 64 else 'pile'}: {k}x{k} random convex polygons, U={U:g}")
    if name.startswith("mix"):   # small mixed scene with circles, for parity tests
        k = int(name[3:]) if len(name) > 3 else 8
        U = 6.0
        rng = np.random.default_rng(77 + k)
        b = Bodies()
        add_walls(b, U)
        for row in range(k):
            for col in range(k):
                x = 0.5 * U + (col - (k - 1) / 2) * 0.32 + float(rng.uniform(-0.03, 0.03))
                y = U - 0.4 - row * 0.3
                mass = max(0.1, float(rng.normal(1.0, 0.1)))
                if rng.uniform() < 0.3:
                    r = float(rng.uniform(0.08, 0.16))
                    b.add(x=x, y=y, vx=float(rng.uniform(-1, 1)), vy=float(rng.uniform(0, 2)),
                          mass=mass, circle=True, radius=r, has_angvel=True, has_inertia=True,
                          inertia=0.5 * mass * r * r, omega=float(rng.uniform(-1, 1)))
                else:
                    verts = regular_polygon(int(rng.integers(3, 9)), float(rng.uniform(0.1, 0.18)))
                    b.add(x=x, y=y, vx=float(rng.uniform(-1, 1)), vy=float(rng.uniform(0, 2)),
                          mass=mass, verts=verts, angle=float(rng.uniform(0, 6.28)),
                          has_angvel=True, has_inertia=True, omega=float(rng.uniform(-1, 1)),
                          inertia=polygon_inertia(verts, mass))
        return dict(U=U, bodies=b, pgs_iterations=10, desc=f"mix: {k}x{k} circles+polygons, U=6")
    raise KeyError(name)


def particles_aos(fl) -> np.ndarray:
    """GPUFluidParticle array as gatherFluidParticles builds it (fluid.cpp:282-295)."""
    from_keys = ("x", "y", "vx", "vy")
    n = len(fl["x"])
    p = np.zeros((n, 13), np.float32)
    for k, name in enumerate(from_keys):
        p[:, k] = fl[name].astype(np.float32)
    p[:, 4] = p[:, 2]
    p[:, 5] = p[:, 3]
    p[:, 8] = fl["mass"].astype(np.float32)
    p[:, 9] = 0.05
    p[:, 10] = 1000.0
    p[:, 11] = fl["density"].astype(np.float32)
    p[:, 12] = fl["pressure"].astype(np.float32)
    return p


# ---------------------------------------------------------------------------
# Barnes-Hut scenes.  The reference's BH scenario is
# KeplerianDiskScenario (src/scenarios/keplerian_disk.cpp:16-31, :45-140,
# include/scenarios/keplerian_disk.hpp:15-42): a 1e36 kg central body at the
# centre of a U = 600 px * 1e7 m/px universe, disk bodies between 100 px and
# 240 px (ScreenLength / outerRadiusFactor) with ~1e22 kg masses falling off as
# (r_min / r)^0.5 and Keplerian speeds, softener 2e7 m.  Seeded synthetic
# version (the reference seeds with time(nullptr)); `n` bodies in total.
BH_MPP = 1e7
BH_U = 600 * BH_MPP
BH_SOFT = 2e7
BH_G = 6.674e-11


def bh_disk(n: int = 1000, seed: int = 11, central_mass: float = 1e36, thin: float = 0.02):
    rng = np.random.default_rng(seed)
    cx = cy = 0.5 * BH_U
    rmin, rmax = 100 * BH_MPP, 240 * BH_MPP
    k = n - 1
    r = rmin + (rmax - rmin) * np.sqrt(rng.random(k))
    ang = rng.random(k) * 2 * math.pi
    x = cx + r * np.cos(ang)
    y = cy + r * np.sin(ang) + rng.normal(0.0, thin * r)
    speed = np.sqrt(BH_G * central_mass / r) * rng.normal(1.0, 0.01, k)
    vx = -speed * np.sin(ang)
    vy = speed * np.cos(ang)
    m = rng.normal((rmin / r) ** 0.5 * 1e22, 1e21)
    return dict(x=np.concatenate([[cx], x]), y=np.concatenate([[cy], y]),
                vx=np.concatenate([[0.0], vx]), vy=np.concatenate([[0.0], vy]),
                m=np.concatenate([[central_mass], m]), U=BH_U, softener=BH_SOFT)


def bh_clustered(n: int = 4096, seed: int = 3, U: float = 1.0e6):
    """Gaussian clusters (deep, unbalanced subtrees), a few bodies outside
    [0, U) (not inserted, still attracted), masses spanning the small-mass
    threshold (1e3) so that all-small nodes are skipped."""
    rng = np.random.default_rng(seed)
    centres = rng.random((8, 2)) * U
    c = rng.integers(0, 8, n)
    pts = centres[c] + rng.normal(0.0, U * 0.01, (n, 2)) * rng.choice([1.0, 0.05], (n, 1))
    pts[: max(1, n // 200)] = rng.random((max(1, n // 200), 2)) * U * 1.5 - 0.25 * U
    m = 10.0 ** rng.uniform(1.0, 9.0, n)
    v = rng.normal(0.0, 1.0, (n, 2))
    return dict(x=pts[:, 0].copy(), y=pts[:, 1].copy(), vx=v[:, 0].copy(), vy=v[:, 1].copy(), m=m, U=U,
                softener=0.0)
