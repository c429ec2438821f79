"""ctypes binding of the MI355X backend's C ABI (include/lpe.h).

This is the Python-side caller used by tests/ and bench.py.  The production
caller is the C++ host mirror under host/ (Systems::FluidSystem & co.), which
binds the same symbols.  The library is the in-tree liblpe_hip.so; there is no
fallback: if it is missing or has no device, calls fail loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

# Hardware queues: a context runs four streams (the fluid step, the
# prelaunch, the collision detection, the position solver), which HIP maps
# round robin onto GPU_MAX_HW_QUEUES queues -- HIP's default of 4 gives each
# its own.  More than 4 measured the kernels ~2x slower on MI355X (ROCm 7.2,
# profiles/r06/hwq/sweep.txt: 810 ticks/s at 4 queues, 453 at 5-8), so the
# binding leaves the variable alone (round 4 set 8 here).

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LPE_LIB") or os.path.join(HERE, "liblpe_hip.so")   # LPE_LIB: an alternative build (A/B runs)

LPE_OK = 0
STATUS = {0: "OK", 1: "ERR_HIP", 2: "ERR_ARG", 3: "ERR_STATE", 4: "ERR_CAPACITY",
          5: "ERR_OVERFLOW", 6: "ERR_NO_DEVICE"}
MAX_POLY_VERTS = 16


class LpeError(RuntimeError):
    pass


# --------------------------------------------------------------------------
# struct mirrors (include/lpe.h)
class _PosSolver(C.Structure):
    _fields_ = [(n, C.c_float) for n in (
        "safetyMargin", "relaxFactor", "maxCorrection", "maxVelocityUpdate",
        "minSafeDistance", "velocityDamping", "minPositionChange")]


class _ImpSolver(C.Structure):
    _fields_ = [(n, C.c_float) for n in (
        "maxForce", "maxTorque", "fluidForceScale", "fluidForceMax", "buoyancyStrength",
        "viscosityScale", "depthScale", "depthTransitionRate", "depthEstimateScale",
        "pressureForceRatio", "viscousForceRatio", "angularDampingThreshold",
        "angularDampingFactor", "maxSafeVelocitySq", "minPenetration", "minRelVelocity")]


class _GridCfg(C.Structure):
    _fields_ = [(n, C.c_float) for n in ("gridEpsilon", "smoothingLength", "boundaryOffset")]


class _NumCfg(C.Structure):
    _fields_ = [(n, C.c_float) for n in (
        "minDistanceThreshold", "minDensityThreshold", "minTimestep", "fallbackTimestep")]


class FluidConfig(C.Structure):
    """Mirror of Systems::FluidConfig (fluid.hpp:131-200)."""
    _fields_ = [("gravity", C.c_float), ("restDensity", C.c_float), ("stiffness", C.c_float),
                ("viscosity", C.c_float), ("positionSolver", _PosSolver),
                ("impulseSolver", _ImpSolver), ("gridConfig", _GridCfg),
                ("numericalConfig", _NumCfg), ("dampingFactor", C.c_float),
                ("numSubSteps", C.c_int), ("threadsPerGroup", C.c_int)]


class RigidStats(C.Structure):
    _fields_ = [("pairs", C.c_int32), ("contacts", C.c_int32), ("pgsLevels", C.c_int32),
                ("posLevels", C.c_int32), ("overflow", C.c_int32), ("colourRounds", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class SphStats(C.Structure):
    _fields_ = [("maxCellOccupancy", C.c_int32), ("notInserted", C.c_int32),
                ("capacityOverflow", C.c_int32), ("listOverflow", C.c_int32),
                ("gridDimX", C.c_int32), ("gridDimY", C.c_int32),
                ("gridMinX", C.c_int32), ("gridMinY", C.c_int32), ("cellSize", C.c_float),
                ("nlistOverflow", C.c_int32), ("rigidCandidates", C.c_int32), ("neighbours", C.c_int32),
                ("stageFallback", C.c_int32), ("overCapCells", C.c_int32), ("refUndefined", C.c_int32),
                ("overCapCellsTotal", C.c_int32), ("maxCellOccupancyTotal", C.c_int32),
                ("haloWire", C.c_int32 * 2), ("slabOwned", C.c_int32), ("slabSlots", C.c_int32),
                ("ghostsIn", C.c_int32 * 2), ("forcesGlobal", C.c_int32),
                ("gridRegrows", C.c_int32), ("slotRegrows", C.c_int32), ("deviceGrid", C.c_int32 * 4)]

    def as_dict(self):
        return {k: (list(getattr(self, k)) if k in ("haloWire", "ghostsIn", "deviceGrid") else getattr(self, k))
                for k, _ in self._fields_}


# numpy mirror of lpe_gpu_rigid / Systems::GPURigidBody (fluid.hpp:94-125), 200 B
RIGID_DTYPE = np.dtype([
    ("shapeType", "<i4"), ("posX", "<f4"), ("posY", "<f4"), ("angle", "<f4"), ("radius", "<f4"),
    ("vertCount", "<i4"), ("vertsX", "<f4", (MAX_POLY_VERTS,)), ("vertsY", "<f4", (MAX_POLY_VERTS,)),
    ("vx", "<f4"), ("vy", "<f4"), ("omega", "<f4"), ("mass", "<f4"), ("inertia", "<f4"),
    ("minX", "<f4"), ("maxX", "<f4"), ("minY", "<f4"), ("maxY", "<f4"),
    ("accumFx", "<f4"), ("accumFy", "<f4"), ("accumTorque", "<f4")])
assert RIGID_DTYPE.itemsize == 200

# numpy mirror of lpe_body (include/lpe.h): one solid body's ECS components
BODY_DTYPE = np.dtype([
    ("eid", "<u4"), ("flags", "<u4"), ("x", "<f8"), ("y", "<f8"), ("angle", "<f8"),
    ("vx", "<f8"), ("vy", "<f8"), ("omega", "<f8"), ("mass", "<f8"), ("inertia", "<f8"),
    ("radius", "<f8"), ("vert_off", "<i4"), ("vert_cnt", "<i4"), ("sleep_counter", "<i4"),
    ("pad", "<i4")])
assert BODY_DTYPE.itemsize == 96
CONTACT_DTYPE = np.dtype([("a", "<i4"), ("b", "<i4"), ("pair", "<i4"), ("pad", "<i4"),
                          ("nx", "<f8"), ("ny", "<f8"), ("pen", "<f8"), ("px", "<f8"),
                          ("py", "<f8")])
assert CONTACT_DTYPE.itemsize == 56

BODY_HAS_PHASE, BODY_SOLID, BODY_LIQUID, BODY_BOUNDARY = 1, 2, 4, 8
BODY_HAS_SLEEP, BODY_ASLEEP, BODY_HAS_ANGPOS, BODY_HAS_ANGVEL = 16, 32, 64, 128
BODY_HAS_INERTIA, BODY_CIRCLE, BODY_POLYGON, BODY_HAS_MASS, BODY_HAS_VEL = 256, 512, 1024, 2048, 4096


class RigidConfig(C.Structure):
    """Mirror of lpe_rigid_config (include/lpe.h)."""
    _fields_ = [("universeSize", C.c_double), ("metersPerPixel", C.c_double),
                ("quadtreeCapacity", C.c_int32), ("pgsIterations", C.c_int32),
                ("boundaryBuffer", C.c_double), ("smallParticleThreshold", C.c_double),
                ("frictionCoeff", C.c_float), ("posIterations", C.c_int32),
                ("baumgarte", C.c_double), ("slop", C.c_double), ("gravity", C.c_double),
                ("planetaryMassThreshold", C.c_double), ("angularDamping", C.c_double),
                ("maxAngularSpeed", C.c_double), ("marginPixels", C.c_double),
                ("bounceDamping", C.c_double), ("maxSpeed", C.c_double),
                ("linearSleepThreshold", C.c_double), ("angularSleepThreshold", C.c_double),
                ("sleepFramesThreshold", C.c_int32), ("pgsMode", C.c_int32)]


PGS_GAUSS_SEIDEL, PGS_JACOBI = 0, 1     # lpe_rigid_config.pgsMode


def rigid_config(universe=6.0, pgs_iterations=10, **kw) -> RigidConfig:
    """Reference defaults (broadphase.hpp, contact_solver.hpp, position_solver.hpp,
    gravity/rotation/boundary/sleep .hpp)."""
    c = RigidConfig(universeSize=universe, metersPerPixel=0.01, quadtreeCapacity=8,
                    pgsIterations=pgs_iterations, boundaryBuffer=500.0,
                    smallParticleThreshold=0.01, frictionCoeff=0.5, posIterations=10,
                    baumgarte=0.02, slop=0.001, gravity=9.8, planetaryMassThreshold=1e10,
                    angularDamping=0.98, maxAngularSpeed=20.0, marginPixels=15.0,
                    bounceDamping=0.7, maxSpeed=1.0, linearSleepThreshold=0.5,
                    angularSleepThreshold=0.5, sleepFramesThreshold=60)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


_FP = C.POINTER(C.c_float)
_IP = C.POINTER(C.c_int32)


def _fp(a):
    if a is None:
        return None
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(_FP)


_lib = None

# every symbol declared in include/lpe.h (checked by tests/test_abi.py)
SIGNATURES = {
    "lpe_abi_version": ([], C.c_int),
    "lpe_device_count": ([_IP], C.c_int),
    "lpe_create": ([C.c_int, C.POINTER(C.c_void_p)], C.c_int),
    "lpe_destroy": ([C.c_void_p], C.c_int),
    "lpe_last_error": ([C.c_void_p], C.c_char_p),
    "lpe_sync": ([C.c_void_p], C.c_int),
    "lpe_hw_queues": ([_IP, _IP], C.c_int),
    "lpe_timing_enable": ([C.c_void_p, C.c_int], C.c_int),
    "lpe_timing_reset": ([C.c_void_p], C.c_int),
    "lpe_timing_read": ([C.c_void_p, C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_double),
                         C.POINTER(C.c_long)], C.c_int),
    "lpe_fluid_config_default": ([C.POINTER(FluidConfig)], C.c_int),
    "lpe_sph_set_config": ([C.c_void_p, C.POINTER(FluidConfig)], C.c_int),
    "lpe_sph_upload": ([C.c_void_p, C.c_int] + [_FP] * 7, C.c_int),
    "lpe_sph_upload_rigids": ([C.c_void_p, C.c_int, C.c_void_p], C.c_int),
    "lpe_sph_step": ([C.c_void_p, C.c_double], C.c_int),
    "lpe_sph_download": ([C.c_void_p] + [_FP] * 6, C.c_int),
    "lpe_sph_download_aux": ([C.c_void_p] + [_FP] * 4, C.c_int),
    "lpe_sph_download_rigids": ([C.c_void_p, C.c_void_p, _FP], C.c_int),
    "lpe_sph_get_stats": ([C.c_void_p, C.POINTER(SphStats)], C.c_int),
    "lpe_sph_diag": ([C.c_void_p, C.c_int], C.c_int),
    "lpe_sph_set_mode": ([C.c_void_p, C.c_int], C.c_int),
    "lpe_sph_probe_cells": ([C.c_void_p, _IP, C.POINTER(SphStats)], C.c_int),
    "lpe_sph_probe_density": ([C.c_void_p, _FP, _FP], C.c_int),
    "lpe_rigid_config_default": ([C.POINTER(RigidConfig)], C.c_int),
    "lpe_rigid_set_config": ([C.c_void_p, C.POINTER(RigidConfig)], C.c_int),
    "lpe_rigid_upload": ([C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p], C.c_int),
    "lpe_rigid_step": ([C.c_void_p, C.POINTER(RigidStats)], C.c_int),
    "lpe_rigid_step_ordered": ([C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                                C.POINTER(RigidStats)], C.c_int),
    "lpe_rigid_integrate": ([C.c_void_p, C.c_int, C.c_double, C.c_double], C.c_int),
    "lpe_rigid_download": ([C.c_void_p, C.c_void_p], C.c_int),
    "lpe_rigid_download_contacts": ([C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p,
                                     _IP, _IP], C.c_int),
    "lpe_rigid_download_colours": ([C.c_void_p, C.c_int, _IP, _IP], C.c_int),
    "lpe_rigid_download_impulses": ([C.c_void_p, C.c_int, _FP, _FP, _IP], C.c_int),
    "lpe_rigid_reserve": ([C.c_void_p, C.c_int, C.c_int], C.c_int),
    "lpe_rigid_buffer_info": ([C.c_void_p, _IP, _IP, _IP], C.c_int),
}

class WorldConfig(C.Structure):
    _fields_ = [("secondsPerTick", C.c_double), ("timeAcceleration", C.c_double),
                ("baseTimeAcceleration", C.c_double), ("timeScale", C.c_double)]


SIGNATURES["lpe_world_set_coupling"] = ([C.c_void_p, C.c_int, C.c_void_p], C.c_int)
SIGNATURES["lpe_world_tick"] = ([C.c_void_p, C.POINTER(WorldConfig), C.c_int], C.c_int)

SIGNATURES["lpe_sph_set_slab"] = ([C.c_void_p, C.c_int, C.c_int, _FP, C.c_int, C.c_int], C.c_int)
SIGNATURES["lpe_sph_set_ids"] = ([C.c_void_p, C.c_int, _IP], C.c_int)
SIGNATURES["lpe_sph_set_global_count"] = ([C.c_void_p, C.c_int], C.c_int)
SIGNATURES["lpe_sph_slab_info"] = ([C.c_void_p, C.c_int, _IP, _IP, _IP], C.c_int)
SIGNATURES["lpe_sph_download_owned"] = ([C.c_void_p, C.c_int] + [_FP] * 6 + [_IP, _IP], C.c_int)
SIGNATURES["lpe_sph_set_domain"] = ([C.c_void_p] + [C.c_double] * 4, C.c_int)
SIGNATURES["lpe_mg_unique_id"] = ([C.c_char_p], C.c_int)
SIGNATURES["lpe_mg_init_rccl"] = ([C.c_void_p, C.c_int, C.c_int, C.c_char_p], C.c_int)
SIGNATURES["lpe_mg_info"] = ([C.c_void_p, _IP, _IP, _IP], C.c_int)
HALO_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_void_p,
                      C.c_size_t, C.c_void_p, C.c_size_t)
REDF_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_float), C.c_int, C.c_int)
REDI_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_longlong), C.c_int)


class HostTransport(C.Structure):
    """lpe_host_transport: the callbacks of the host-staged slab transport."""
    _fields_ = [("user", C.c_void_p), ("halo", HALO_FN), ("allreduce_f32", REDF_FN), ("allreduce_i64", REDI_FN)]


SIGNATURES["lpe_mg_init_host"] = ([C.c_void_p, C.c_int, C.c_int, C.POINTER(HostTransport)], C.c_int)
SIGNATURES["lpe_mg_loopback_run"] = ([C.c_int, C.POINTER(C.c_void_p), C.POINTER(WorldConfig), C.c_double,
                                      C.c_int], C.c_int)

class RenderParams(C.Structure):
    _fields_ = [("gridW", C.c_int32), ("gridH", C.c_int32), ("cellSize", C.c_float),
                ("originX", C.c_float), ("originY", C.c_float), ("smoothingRadius", C.c_float)]


SIGNATURES["lpe_render_density"] = ([C.c_void_p, C.POINTER(RenderParams), _FP, _FP], C.c_int)

class BhConfig(C.Structure):
    """lpe_bh_config: BarnesHutConfig (barnes_hut.hpp:19-25) + the shared fields it reads."""
    _fields_ = [("theta", C.c_double), ("small_mass_threshold", C.c_double), ("universe_size", C.c_double),
                ("softener", C.c_double), ("G", C.c_double)]


class BhStats(C.Structure):
    _fields_ = [("skipped", C.c_int32), ("inserted", C.c_int32), ("nodes", C.c_int32), ("depth", C.c_int32)]

    def as_dict(self):
        return {k: int(getattr(self, k)) for k, _ in self._fields_}


_DP = C.POINTER(C.c_double)
SIGNATURES["lpe_bh_config_default"] = ([C.POINTER(BhConfig)], C.c_int)
SIGNATURES["lpe_bh_upload"] = ([C.c_void_p, C.c_int] + [_DP] * 5 + [C.c_void_p], C.c_int)
SIGNATURES["lpe_bh_step"] = ([C.c_void_p, C.POINTER(BhConfig), C.c_double, C.POINTER(BhStats)], C.c_int)
SIGNATURES["lpe_bh_download"] = ([C.c_void_p, _DP, _DP], C.c_int)
SIGNATURES["lpe_world_set_barnes_hut"] = ([C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_void_p], C.c_int)


def bh_config(universe: float, theta: float = 0.5, small_mass_threshold: float = 1e3,
              softener: float = 0.0) -> BhConfig:
    cfg = BhConfig()
    lib().lpe_bh_config_default(C.byref(cfg))
    cfg.universe_size = universe
    cfg.theta = theta
    cfg.small_mass_threshold = small_mass_threshold
    cfg.softener = softener
    return cfg


SYS_BOUNDARY, SYS_GRAVITY, SYS_ROTATION, SYS_MOVEMENT, SYS_SLEEP = 1, 2, 4, 8, 16
SPH_MODE_REF_CELL_CAP = 1       # LPE_SPH_MODE_REF_CELL_CAP (include/lpe.h)
SPH_MODE_PROBE_TICK_PASS = 2    # LPE_SPH_MODE_PROBE_TICK_PASS


ABI_VERSION = 2                 # LPE_ABI_VERSION of include/lpe.h


def lib():
    """Load the in-tree HIP library (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LpeError(f"{LIB_PATH} not built: run `make` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        if L.lpe_abi_version() != ABI_VERSION:
            raise LpeError(f"{LIB_PATH}: ABI version {L.lpe_abi_version()}, this binding needs {ABI_VERSION} "
                           "(rebuild with `make`)")
        _lib = L
    return _lib


def default_fluid_config() -> FluidConfig:
    cfg = FluidConfig()
    lib().lpe_fluid_config_default(C.byref(cfg))
    return cfg


def mg_unique_id() -> bytes:
    """128-byte RCCL unique id (rank 0 makes it, every rank passes it to mg_init_rccl)."""
    buf = C.create_string_buffer(128)
    st = lib().lpe_mg_unique_id(buf)
    if st != LPE_OK:
        raise LpeError(f"lpe_mg_unique_id: {STATUS.get(st, st)}")
    return buf.raw


def mg_loopback_run(ctxs, nticks: int, dt_tick: float = 0.0, world: "WorldConfig" = None):
    """Advance the contexts (ranks 0..n-1 of an in-process slab group) nticks."""
    arr = (C.c_void_p * len(ctxs))(*[c._h.value for c in ctxs])
    st = lib().lpe_mg_loopback_run(len(ctxs), arr, C.byref(world) if world is not None else None,
                                   float(dt_tick), int(nticks))
    if st != LPE_OK:
        msgs = [lib().lpe_last_error(c._h) for c in ctxs]
        raise LpeError(f"lpe_mg_loopback_run: {STATUS.get(st, st)}: "
                       + "; ".join(m.decode() for m in msgs if m))


def hw_queues() -> dict:
    """GPU_MAX_HW_QUEUES in effect (lpe_hw_queues) and whether the library set it."""
    q, by = C.c_int32(0), C.c_int32(0)
    lib().lpe_hw_queues(C.byref(q), C.byref(by))
    return dict(queues=q.value, set_by_library=bool(by.value))


def device_count() -> int:
    c = C.c_int32(0)
    lib().lpe_device_count(C.byref(c))
    return c.value


class Context:
    """One lpe_ctx (one HIP device + stream)."""

    def __init__(self, device: int = 0):
        self._h = C.c_void_p()
        st = lib().lpe_create(device, C.byref(self._h))
        if st != LPE_OK:
            raise LpeError(f"lpe_create(device={device}) failed: {STATUS.get(st, st)}")
        self.n = 0
        self.nr = 0

    def close(self):
        if self._h:
            lib().lpe_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, st, what):
        if st != LPE_OK:
            msg = lib().lpe_last_error(self._h)
            raise LpeError(f"{what}: {STATUS.get(st, st)}: {msg.decode() if msg else ''}")

    def sync(self):
        self._chk(lib().lpe_sync(self._h), "lpe_sync")

    # ---- kernel timing -------------------------------------------------
    def timing(self, on=True):
        """on: False/0 off, True/1 every kernel, 2 the dominant kernels only."""
        self._chk(lib().lpe_timing_enable(self._h, int(on)), "lpe_timing_enable")

    def timing_reset(self):
        self._chk(lib().lpe_timing_reset(self._h), "lpe_timing_reset")

    def timing_read(self) -> dict:
        """{kernel_name: (total_ms, calls)} accumulated since the last reset."""
        out = {}
        i = 0
        buf = C.create_string_buffer(128)
        while True:
            ms = C.c_double(0)
            calls = C.c_long(0)
            st = lib().lpe_timing_read(self._h, i, buf, 128, C.byref(ms), C.byref(calls))
            if st != LPE_OK:
                break
            out[buf.value.decode()] = (ms.value, calls.value)
            i += 1
        return out

    # ---- SPH -----------------------------------------------------------
    def sph_set_config(self, cfg: FluidConfig):
        self._chk(lib().lpe_sph_set_config(self._h, C.byref(cfg)), "lpe_sph_set_config")

    def sph_upload(self, x, y, vx, vy, m, density=None, pressure=None):
        arrs = [np.ascontiguousarray(a, dtype=np.float32) if a is not None else None
                for a in (x, y, vx, vy, m, density, pressure)]
        self._keep = arrs
        self.n = int(arrs[0].shape[0])
        self._chk(lib().lpe_sph_upload(self._h, self.n, *[_fp(a) for a in arrs]), "lpe_sph_upload")

    def sph_upload_rigids(self, rigids):
        r = np.ascontiguousarray(rigids, dtype=RIGID_DTYPE)
        self.nr = int(r.shape[0])
        self._chk(lib().lpe_sph_upload_rigids(self._h, self.nr, r.ctypes.data if self.nr else None),
                  "lpe_sph_upload_rigids")

    def sph_step(self, dt_tick: float):
        self._chk(lib().lpe_sph_step(self._h, float(dt_tick)), "lpe_sph_step")

    def sph_download(self):
        out = {k: np.empty(self.n, np.float32) for k in ("x", "y", "vx", "vy", "density", "pressure")}
        self._chk(lib().lpe_sph_download(self._h, *[_fp(out[k]) for k in
                  ("x", "y", "vx", "vy", "density", "pressure")]), "lpe_sph_download")
        aux = {k: np.empty(self.n, np.float32) for k in ("vxHalf", "vyHalf", "ax", "ay")}
        self._chk(lib().lpe_sph_download_aux(self._h, *[_fp(aux[k]) for k in
                  ("vxHalf", "vyHalf", "ax", "ay")]), "lpe_sph_download_aux")
        out.update(aux)
        return out

    def sph_download_rigids(self):
        r = np.zeros(self.nr, RIGID_DTYPE)
        acc = np.zeros(3 * max(self.nr, 1), np.float32)
        self._chk(lib().lpe_sph_download_rigids(self._h, r.ctypes.data if self.nr else None,
                                                _fp(acc)), "lpe_sph_download_rigids")
        return r, acc[:3 * self.nr].reshape(-1, 3)

    def sph_stats(self) -> dict:
        s = SphStats()
        self._chk(lib().lpe_sph_get_stats(self._h, C.byref(s)), "lpe_sph_get_stats")
        return s.as_dict()

    def sph_set_mode(self, flags: int):
        """LPE_SPH_MODE_* flags (SPH_MODE_REF_CELL_CAP: the reference's 64-slot cells)."""
        self._chk(lib().lpe_sph_set_mode(self._h, int(flags)), "lpe_sph_set_mode")

    def sph_diag(self, on=True):
        self._chk(lib().lpe_sph_diag(self._h, int(on)), "lpe_sph_diag")

    # ---- x-slab decomposition --------------------------------------------
    def sph_set_slab(self, nranks, rank, edges, wire_cap, rebalance=0):
        """Slab `rank` of `nranks`: edges (nranks + 1 metres, inner ones on
        reference-cell boundaries), wire_cap ghost records per direction and
        sub-step, rebalance > 0: move the edges every that many fluid steps."""
        e = np.ascontiguousarray(edges, np.float32)
        assert len(e) == nranks + 1
        self._slab_edges = e
        self._chk(lib().lpe_sph_set_slab(self._h, int(nranks), int(rank), _fp(e), int(wire_cap), int(rebalance)),
                  "lpe_sph_set_slab")

    def sph_slab_info(self) -> dict:
        """{nranks, mv, edges}: the slab rank's current edges in reference-cell
        columns (re-balancing moves them) and how far they may move."""
        nr, mv = C.c_int(0), C.c_int(0)
        self._chk(lib().lpe_sph_slab_info(self._h, 0, None, C.byref(nr), C.byref(mv)), "lpe_sph_slab_info")
        e = np.zeros(max(nr.value + 1, 1), np.int32)
        self._chk(lib().lpe_sph_slab_info(self._h, len(e), e.ctypes.data_as(_IP), C.byref(nr), C.byref(mv)),
                  "lpe_sph_slab_info")
        return dict(nranks=nr.value, mv=mv.value, edges=e[:nr.value + 1])

    def sph_set_ids(self, ids):
        a = np.ascontiguousarray(ids, dtype=np.int32)
        self._chk(lib().lpe_sph_set_ids(self._h, len(a), a.ctypes.data_as(_IP)), "lpe_sph_set_ids")

    def sph_set_global_count(self, n_global: int):
        self._chk(lib().lpe_sph_set_global_count(self._h, int(n_global)), "lpe_sph_set_global_count")

    def sph_download_owned(self, cap=None):
        """{x, y, vx, vy, density, pressure, id} of the particles this context owns."""
        n = C.c_int(0)
        cap = int(cap if cap is not None else max(self.n, 1))
        while True:
            out = {k: np.empty(cap, np.float32) for k in ("x", "y", "vx", "vy", "density", "pressure")}
            ids = np.empty(cap, np.int32)
            st = lib().lpe_sph_download_owned(self._h, cap, *[_fp(out[k]) for k in
                                              ("x", "y", "vx", "vy", "density", "pressure")],
                                              ids.ctypes.data_as(_IP), C.byref(n))
            if st == 4 and n.value > cap:  # LPE_ERR_CAPACITY
                cap = n.value
                continue
            self._chk(st, "lpe_sph_download_owned")
            break
        k = n.value
        out = {key: v[:k] for key, v in out.items()}
        out["id"] = ids[:k]
        return out

    def sph_set_domain(self, x0, y0, x1, y1):
        self._chk(lib().lpe_sph_set_domain(self._h, float(x0), float(y0), float(x1), float(y1)),
                  "lpe_sph_set_domain")

    def render_density(self, grid_w, grid_h, cell_size=0.01, origin=(0.0, 0.0), smoothing_radius=10.0,
                       download=True):
        """FluidRenderer's density field: (normalised grid [grid_h, grid_w], max)."""
        p = RenderParams(int(grid_w), int(grid_h), float(cell_size), float(origin[0]), float(origin[1]),
                         float(smoothing_radius))
        out = np.empty((int(grid_h), int(grid_w)), np.float32) if download else None
        mx = np.zeros(1, np.float32)
        self._chk(lib().lpe_render_density(self._h, C.byref(p), _fp(out.reshape(-1)) if download else None,
                                           _fp(mx)), "lpe_render_density")
        return out, float(mx[0])

    def mg_init_rccl(self, nranks: int, rank: int, uid: bytes):
        assert len(uid) == 128
        self._chk(lib().lpe_mg_init_rccl(self._h, int(nranks), int(rank), uid), "lpe_mg_init_rccl")

    def mg_info(self) -> dict:
        """{nranks, rank, comm_ranks}: the transport's group; comm_ranks is what
        the communicator itself reports (ncclCommCount for RCCL)."""
        a, b, c = C.c_int32(0), C.c_int32(0), C.c_int32(0)
        self._chk(lib().lpe_mg_info(self._h, C.byref(a), C.byref(b), C.byref(c)), "lpe_mg_info")
        return dict(nranks=a.value, rank=b.value, comm_ranks=c.value)

    def mg_init_host(self, nranks: int, rank: int, transport):
        """Host-staged transport: `transport` has halo(sendL, sendR, recvL,
        recvR) over numpy uint8 views (None where there is no neighbour),
        allreduce_f32(arr, op) and allreduce_i64(arr), each reducing in place
        and raising on failure (slab.GlooTransport is the torch.distributed
        one).  The callbacks stay referenced by this context."""
        def view(ptr, n, ct):
            return None if not ptr or n == 0 else np.ctypeslib.as_array((ct * n).from_address(ptr))

        def halo(_u, sL, nsL, sR, nsR, rL, nrL, rR, nrR):
            try:
                transport.halo(view(sL, nsL, C.c_uint8), view(sR, nsR, C.c_uint8),
                               view(rL, nrL, C.c_uint8), view(rR, nrR, C.c_uint8))
                return 0
            except Exception as e:       # noqa: BLE001  (no exception may cross the C boundary)
                transport.last_error = repr(e)
                return 1

        def redf(_u, buf, n, op):
            try:
                transport.allreduce_f32(np.ctypeslib.as_array(buf, shape=(n,)), int(op))
                return 0
            except Exception as e:       # noqa: BLE001
                transport.last_error = repr(e)
                return 1

        def redi(_u, buf, n):
            try:
                transport.allreduce_i64(np.ctypeslib.as_array(buf, shape=(n,)))
                return 0
            except Exception as e:       # noqa: BLE001
                transport.last_error = repr(e)
                return 1

        t = HostTransport(None, HALO_FN(halo), REDF_FN(redf), REDI_FN(redi))
        self._host_transport = (t, transport)
        self._chk(lib().lpe_mg_init_host(self._h, int(nranks), int(rank), C.byref(t)), "lpe_mg_init_host")

    def sph_probe_cells(self):
        cells = np.empty(self.n, np.int32)
        s = SphStats()
        self._chk(lib().lpe_sph_probe_cells(self._h, cells.ctypes.data_as(_IP), C.byref(s)),
                  "lpe_sph_probe_cells")
        return cells, s.as_dict()

    # ---- rigid ----------------------------------------------------------
    def rigid_set_config(self, cfg: "RigidConfig"):
        self._chk(lib().lpe_rigid_set_config(self._h, C.byref(cfg)), "lpe_rigid_set_config")

    def rigid_upload(self, bodies, verts):
        b = np.ascontiguousarray(bodies, dtype=BODY_DTYPE)
        v = np.ascontiguousarray(verts, dtype=np.float64).reshape(-1)
        self.nb = len(b)
        self._rkeep = (b, v)
        self._chk(lib().lpe_rigid_upload(self._h, len(b), b.ctypes.data, len(v) // 2, v.ctypes.data),
                  "lpe_rigid_upload")

    def rigid_step(self, pairs=None, pgs_order=None, stats=True):
        st = RigidStats()
        if pairs is None and pgs_order is None:
            r = lib().lpe_rigid_step(self._h, C.byref(st) if stats else None)
        else:
            p = np.ascontiguousarray(pairs, np.int32).reshape(-1)
            o = None if pgs_order is None else np.ascontiguousarray(pgs_order, np.int32)
            r = lib().lpe_rigid_step_ordered(self._h, len(p) // 2, p.ctypes.data if len(p) else None,
                                             0 if o is None else len(o),
                                             None if o is None else o.ctypes.data,
                                             C.byref(st) if stats else None)
        self._chk(r, "lpe_rigid_step")
        return st.as_dict()

    def rigid_reserve(self, pairs: int, contacts: int):
        self._chk(lib().lpe_rigid_reserve(self._h, int(pairs), int(contacts)), "lpe_rigid_reserve")

    def rigid_buffer_info(self) -> dict:
        p, c, r = C.c_int32(0), C.c_int32(0), C.c_int32(0)
        self._chk(lib().lpe_rigid_buffer_info(self._h, C.byref(p), C.byref(c), C.byref(r)),
                  "lpe_rigid_buffer_info")
        return dict(pairs=p.value, contacts=c.value, regrows=r.value)

    def rigid_integrate(self, systems, dt_state, dt_move=None):
        self._chk(lib().lpe_rigid_integrate(self._h, int(systems), float(dt_state),
                                            float(dt_state if dt_move is None else dt_move)),
                  "lpe_rigid_integrate")

    def rigid_download(self):
        b = np.zeros(self.nb, BODY_DTYPE)
        self._chk(lib().lpe_rigid_download(self._h, b.ctypes.data), "lpe_rigid_download")
        return b

    def rigid_contacts(self):
        np_ = C.c_int32(0)
        nc = C.c_int32(0)
        self._chk(lib().lpe_rigid_download_contacts(self._h, 0, None, 0, None, C.byref(np_),
                                                    C.byref(nc)), "lpe_rigid_download_contacts")
        pairs = np.zeros(2 * max(np_.value, 1), np.int32)
        cs = np.zeros(max(nc.value, 1), CONTACT_DTYPE)
        self._chk(lib().lpe_rigid_download_contacts(self._h, np_.value, pairs.ctypes.data, nc.value,
                                                    cs.ctypes.data, C.byref(np_), C.byref(nc)),
                  "lpe_rigid_download_contacts")
        return pairs[:2 * np_.value].reshape(-1, 2), cs[:nc.value]

    def rigid_colours(self):
        """(pair colours of the last canonical step, colour count)."""
        n = C.c_int32(0)
        self._chk(lib().lpe_rigid_download_colours(self._h, 0, None, C.byref(n)),
                  "lpe_rigid_download_colours")
        np_ = C.c_int32(0)
        self._chk(lib().lpe_rigid_download_contacts(self._h, 0, None, 0, None, C.byref(np_), None),
                  "lpe_rigid_download_contacts")
        col = np.zeros(max(np_.value, 1), np.int32)
        self._chk(lib().lpe_rigid_download_colours(self._h, np_.value, col.ctypes.data_as(_IP),
                                                   C.byref(n)), "lpe_rigid_download_colours")
        return col[:np_.value], n.value

    def rigid_impulses(self):
        """(lamN, lamF) of the last step's contact solve, in rigid_contacts order."""
        n = C.c_int32(0)
        self._chk(lib().lpe_rigid_download_impulses(self._h, 0, None, None, C.byref(n)),
                  "lpe_rigid_download_impulses")
        ln = np.zeros(n.value, np.float32)
        lf = np.zeros(n.value, np.float32)
        self._chk(lib().lpe_rigid_download_impulses(self._h, n.value, _fp(ln), _fp(lf), C.byref(n)),
                  "lpe_rigid_download_impulses")
        return ln, lf

    # ---- world (resident full tick) -------------------------------------
    def world_set_coupling(self, body_index=None):
        if body_index is None:
            self._chk(lib().lpe_world_set_coupling(self._h, -1, None), "lpe_world_set_coupling")
        else:
            idx = np.ascontiguousarray(body_index, np.int32)
            self._ckeep = idx
            self._chk(lib().lpe_world_set_coupling(self._h, len(idx), idx.ctypes.data),
                      "lpe_world_set_coupling")

    def world_tick(self, dt=1.0 / 120.0, nticks=1, time_accel=1.0, bta=1.0, ts=1.0):
        wc = WorldConfig(dt, time_accel, bta, ts)
        self._chk(lib().lpe_world_tick(self._h, C.byref(wc), int(nticks)), "lpe_world_tick")

    def sph_probe_density(self):
        rho = np.empty(self.n, np.float32)
        p = np.empty(self.n, np.float32)
        self._chk(lib().lpe_sph_probe_density(self._h, _fp(rho), _fp(p)), "lpe_sph_probe_density")
        return rho, p

    # ---- Barnes-Hut (lpe_bh_*) ----
    def bh_upload(self, x, y, vx, vy, m, has_vel=None):
        """Bodies in buildTree's insertion order (barnes_hut.cpp:117-128)."""
        a = [np.ascontiguousarray(v, np.float64) for v in (x, y, vx, vy, m)]
        hv = None if has_vel is None else np.ascontiguousarray(has_vel, np.uint8)
        self._bh_keep = (a, hv)
        self.nbh = len(a[0])
        dp = [v.ctypes.data_as(_DP) for v in a]
        self._chk(lib().lpe_bh_upload(self._h, self.nbh, *dp, None if hv is None else hv.ctypes.data),
                  "lpe_bh_upload")

    def bh_step(self, cfg: "BhConfig", dt: float) -> dict:
        st = BhStats()
        self._chk(lib().lpe_bh_step(self._h, C.byref(cfg), float(dt), C.byref(st)), "lpe_bh_step")
        return st.as_dict()

    def bh_download(self):
        vx = np.zeros(self.nbh, np.float64)
        vy = np.zeros(self.nbh, np.float64)
        self._chk(lib().lpe_bh_download(self._h, vx.ctypes.data_as(_DP), vy.ctypes.data_as(_DP)),
                  "lpe_bh_download")
        return vx, vy

    def world_set_barnes_hut(self, enable=True, cfg: "BhConfig" = None, order=None):
        """BarnesHutSystem inside lpe_world_tick (on by default; cfg None: the
        defaults with the rigid config's universe; order None: every massive
        non-boundary body, last first)."""
        o = None if order is None else np.ascontiguousarray(order, np.int32)
        self._bh_world_keep = o
        self._chk(lib().lpe_world_set_barnes_hut(self._h, 1 if enable else 0,
                                                  None if cfg is None else C.byref(cfg),
                                                  0 if o is None else len(o), None if o is None else o.ctypes.data),
                  "lpe_world_set_barnes_hut")
