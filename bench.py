"""bench.py — physics steps/s of the MI355X backend on the metric scene.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scene M]

A step is one tick (ECSSimulator::tick, src/sim.cpp:156-163) of the resident
device pipeline on the scene BASELINE.json's metric is quoted on: M = 256k SPH
particles + 4096 pentagons + 4 walls, synthetic seeded input
already resident in HBM.

For N > 1 (torch.distributed.run, one rank per GPU) the run is weak-scaled
along the SPH path, the path that shards: scene MW{N} is the
M pool widened N times (N x 256k particles, the same 4096-pentagon pile in the
middle, U = 32 N m), its fluid split into N equal-count x-slabs with the RCCL
halo exchange of include/lpe.h, the rigid pass replicated on every rank (rigid
accumulators all-reduced once per tick).  Each rank advances one M-sized SPH
slab per tick, so `value` = N x MW{N} ticks/s: the whole job's throughput in
ticks/s of the 256k-particle metric scene (the contract's whole-job aggregate,
comparable with the N = 1 line).  The same line carries `scaling_weak` (MW{N}
ticks/s, particle-ticks/s, efficiency against scene M as one domain on one
GPU, measured in this run) and `scaling_strong_c5`: north_star's fixed
2M-particle scene C5 over the same N ranks, its single-GPU rate measured in
this run, speedup and efficiency.  Slab ranks and both baselines run
unbounded cells; the all-rank `reference_envelope` says whether the windows
stayed inside the reference's 64-particle cells, where the two cell
semantics are the same computation.  MW1 is M.  --replicas runs N
independent copies of M instead.  The control plane (uid broadcast, barrier,
max over ranks) uses gloo.

Rank 0 prints ONE JSON line (the driver contract), including the live
roofline of the dominant kernel (HIP events on the library's stream) and the
CPU baseline (the oracle on 1 thread and on all cores, on a bounded sample of
the same workload).  Besides the contract window of exactly K ticks (`value`)
the line carries SURVEY.md §8(d)'s methodology: the median of >= 5 windows of
>= 2 s (`windows`), the one-tick-per-call rate of the drop-in path, strict
mode (ECS sync every tick), the BASELINE configs C1-C4 beside the reference's
own measured anchors, and whether the timed window stayed inside the
reference's 64-particle cell capacity.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "little-physics-engine_amd")

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)


def _load(name, path):
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


# Algorithmic (compulsory) bytes per launch, SURVEY.md §8(d) staged model
# (fp32 SoA, per particle per sub-step); C = reference grid cells.
def kernel_bytes(name, n, cells):
    model = {
        "k_kick_drift": 44.0 * n,                    # x,y,vx,vy,ax,ay -> x,y,vh + key
        "k_density": 24.0 * n + 8.0 * cells,         # idx,x,y,m -> rho,p ; cell ranges
        # forces + finish + coupling test, plus the next sub-step's kick fused
        # into 9 of a tick's 10 launches (KickNext): x,y,vx,vy,ax,ay are already
        # in registers, so +16 B kicked state + 4 B key per particle on those
        "k_forces_couple": (40.0 + 24.0 + 8.0 + 0.9 * 20.0) * n,
        "k_scatter": 12.0 * n / 2.0,                 # counting sort (12 B) split over
        "k_rank_permute": 12.0 * n / 2.0,            #   scatter + rank
    }
    return model.get(name)


def lib_sha256():
    """sha256 of the library this run loads (the PMC summaries record the one they profiled)."""
    import hashlib
    lpe = _load("lpe", os.path.join(PKG, "lpe.py"))
    try:
        return hashlib.sha256(open(lpe.LIB_PATH, "rb").read()).hexdigest()
    except OSError:
        return None


def _pmc_lookup(fname, kernel, field):
    """(value, source, same_build) from the newest committed profiles/r*/fname
    holding `kernel`; same_build: its recorded library hash equals this run's."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", fname)), reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if kernel in d:
            built = d.get("_build", {}).get("lib_sha256")
            return d[kernel][field], os.path.relpath(path, ROOT), (built is not None and built == lib_sha256())
    return None, None, False


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC
    measurement (profiles/r*/pmc_traffic.json, written by
    profiles/pmc_traffic.py from separate rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes of the settled metric scene), its file, and whether it profiled
    the library this run loads."""
    return _pmc_lookup("pmc_traffic.json", kernel, "hbm_bytes")


# VALU issue peak: 256 CUs x 4 SIMDs x 2.4 GHz, one wave64 instruction per 2
# cycles per SIMD (32 lanes/cycle; MI355X_MICROARCH.md: FP32 vector 157.3 TF =
# 64 flop/clk/SIMD)
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2.0


def pmc_valu(kernel):
    """VALU wave-instructions per launch of `kernel` from the newest committed
    PMC pass (profiles/r*/pmc_valu.json: SQ_INSTS_VALU), its file, same build."""
    return _pmc_lookup("pmc_valu.json", kernel, "valu_wave_insts")


def rocprof_window(kernel):
    """(avg us, source, same_build) of `kernel` from the newest committed
    rocprofv3 kernel trace of the bench command (profiles/r*/rocprof_window.json,
    profiles/rocpd_summary.py --json over the bench's per-kernel timing window)."""
    return _pmc_lookup("rocprof_window.json", kernel, "avg_us")


def dropin_record():
    """The drop-in timed through the reference's own tick loop (the EnTT host
    harness, profiles/dropin_timing.py), from the newest committed
    profiles/r*/dropin.json: ticks/s of strict mode and of resident mode
    synced every 1 / 10 ticks, and whether it timed the library this run
    loads.  It is measured beside the bench (its 3,000-tick settle and three
    host-driven runs take minutes), not inside it."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "dropin.json")), reverse=True):
        try:
            d = json.loads(open(path).read().strip().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        built = d.get("_build", {}).get("lib_sha256")
        runs = {k: dict(ticks_per_s=r["ticks_per_s"], ms_per_tick=r["ms_per_tick"]) for k, r in d.get("runs", {}).items()}
        strict = d.get("runs", {}).get("strict", {})
        return dict(source=os.path.relpath(path, ROOT), same_build=built is not None and built == lib_sha256(),
                    driver=d.get("driver"), runs=runs, strict_fluid_phases_ms_per_tick=strict.get("fluid_phases_ms_per_tick"))
    return None


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(scene_name, state=None, budget_s=20.0):
    """The oracle (C/C++ restatement of the reference algorithms, -O2) running
    the same full tick on the same scene state (`state`: the device state at
    the end of the timed window, so the CPU ticks the settled pile), on one
    thread (the reference's execution model) and on every host core (OpenMP
    over particles; bit-identical results)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # noqa: E402  (checker / baseline only)
    lpe = _load("lpe", os.path.join(PKG, "lpe.py"))
    scenes = _load("scenes", os.path.join(PKG, "scenes.py"))
    s = scenes.scene(scene_name)
    b, v = scenes.to_bodies(s["bodies"])
    fl = dict(s["fluid"])
    if state is not None:
        fl.update({k: state["fluid"][k] for k in ("x", "y", "vx", "vy", "density", "pressure")})
        b = state["bodies"]
    p0 = scenes.particles_aos(fl)
    couple = np.arange(len(b) - 1, -1, -1, dtype=np.int32)
    fcfg = lpe.default_fluid_config()
    rcfg = lpe.rigid_config(universe=s["U"])
    nproc = os.cpu_count() or 1
    # the box exports OMP_NUM_THREADS (its CPU share); os.cpu_count() is the whole machine
    allc = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or nproc

    def run(threads, budget):
        oracle.set_threads(threads)
        p, bb = p0, b
        ticks = 0
        t0 = time.perf_counter()
        while True:
            p, bb = oracle.world_tick(fcfg, rcfg, p, bb, v, couple, 1.0 / 120.0, 1)
            ticks += 1
            el = time.perf_counter() - t0
            if el > budget or el / ticks * (ticks + 1) > budget * 1.5:
                break
        return ticks / el, ticks

    one, n1 = run(1, budget_s)
    many, nm = run(allc, budget_s / 2)
    oracle.set_threads(0)
    return dict(value=one, unit="ticks/s", cores=1, kind="port",
                all_cores=dict(value=many, cores=allc, ticks=nm,
                               label="the GPU box's per-GPU CPU share (OMP_NUM_THREADS threads of "
                                     f"{nproc} hardware threads)" if os.environ.get("OMP_NUM_THREADS")
                                     else "every hardware thread of the host"),
                nproc=nproc, cpu_model=cpu_model(),
                sample=f"{n1} full tick(s) (1 thread) and {nm} (all {allc} threads) of scene {scene_name}"
                       f"{' from the settled device state' if state is not None else ''} ({len(p0)} SPH particles, "
                       f"{len(b)} bodies) through oracle/ (sph_oracle.c + rigid_oracle.cpp lpeo_world_tick), -O2")


def density_microbench(lpe, scenes, device, side=4096, reps=5):
    """SURVEY.md §8(d) density microbench: a side x side lattice (16.7M
    particles at side 4096) in a U = 104 m universe, one density pass from a
    pre-built grid (lpe_sph_probe_density: hash of the current positions,
    then the pass), timed with HIP events on the library's stream;
    algorithmic bytes 24 B/particle + 8 B/cell (§8(d)).  Two passes:
    the pure one (computeDensity's outputs: k_density_plan + k_density_pair,
    two particles per lane, avg_us the SUM of both launches) and, as
    `tick_pass`, the tick's own k_density<true> (which also writes the forces
    pass's neighbour lists, 256 B of list per particle at this size)."""
    rng = np.random.default_rng(7)
    U = 104.0
    x0 = 0.5 * (U - side * scenes.LATTICE_S)
    fl = scenes.fluid_lattice(rng, side, side, x0, x0)
    ctx = lpe.Context(device)
    res = {}
    try:
        ctx.sph_set_config(lpe.default_fluid_config())
        ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        del fl
        for tag, mode in (("pure", 0), ("tick", lpe.SPH_MODE_PROBE_TICK_PASS)):
            ctx.sph_set_mode(mode)
            rho, _ = ctx.sph_probe_density()          # warm (code objects, caches)
            ctx.sph_diag(True)                        # resets the stage-fallback counter
            ctx.timing(2)
            ctx.timing_reset()
            for _ in range(reps):
                rho, _ = ctx.sph_probe_density()
            tr = ctx.timing_read()
            ctx.timing(0)
            st = ctx.sph_stats()
            res[tag] = (tr, st, float(np.mean(rho)))
        ctx.sph_set_mode(0)
    finally:
        ctx.close()
    n = side * side
    out = None
    for tag in ("pure", "tick"):
        tr, st, mean_rho = res[tag]
        t = tr.get("k_density")
        tp = tr.get("k_density_plan", (0.0, 0))       # the pure pass's per-tile staging plans (its own launch)
        cells = st["gridDimX"] * st["gridDimY"]
        avg_s = (t[0] + tp[0]) / max(t[1], 1) / 1e3
        b = 24.0 * n + 8.0 * cells
        ach = b / avg_s / 1e9
        d = dict(kernel="k_density_pair" if tag == "pure" else "k_density<true>", particles=n, cells=cells,
                 avg_us=round(avg_s * 1e6, 1),
                 kernels_us={"k_density_plan": round(tp[0] / max(tp[1], 1) * 1e3, 1),
                             "k_density": round(t[0] / max(t[1], 1) * 1e3, 1)},
                 algorithmic_bytes=b, achieved=round(ach, 1), unit="GB/s", peak=HBM_PEAK_GBS,
                 frac=round(ach / HBM_PEAK_GBS, 4), launches=t[1],
                 stage_fallback_blocks=st["stageFallback"] // max(reps, 1),
                 mean_density=mean_rho, max_cell_occupancy=st["maxCellOccupancy"])
        if tag == "pure":
            out = d
        else:
            out["tick_pass"] = d
    return out


def render_bench(ctx, U, reps=3):
    """The screen-space fluid density field (lpe_render_density, SURVEY.md
    §8(f) rank 3) of the settled scene: the renderer's own parameters
    (fluid_renderer.cpp:368-388: one cell per pixel at MetersPerPixel = 0.01,
    origin (0, 0), smoothingRadius 10), over the whole U x U universe."""
    side = int(round(U / 0.01))
    ctx.render_density(side, side, 0.01, (0.0, 0.0), 10.0, download=False)      # warm
    ctx.timing(1)
    ctx.timing_reset()
    for _ in range(reps):
        _, mx = ctx.render_density(side, side, 0.01, (0.0, 0.0), 10.0, download=False)
    t = ctx.timing_read()
    ctx.timing(0)
    keys = ("k_render_density", "k_box_blur", "k_grid_max", "k_normalize_density")
    frame = sum(t[k][0] for k in t) / reps * 1e3
    return dict(cells=side * side, kernels_us={k: round(t[k][0] / max(t[k][1], 1) * 1e3, 1) for k in keys if k in t},
                frame_kernels_us=round(frame, 1), max_density=mx,
                note="includes the hash of the current positions (k_kick_drift probe, scan, scatter, permute)")


def loopback_check(args, lpe, scenes, slab, device):
    """K slab ranks of MW{K} (or of C5 with --scene C5) on one GPU through the
    in-process transport (stream-ordered like RCCL: the host never waits for
    the device), beside the same scene as ONE domain on the same GPU: the
    ratio of the two walls is the decomposition's overhead (ghost work,
    exchanges, the extra launches), since both do the same physics on the
    same GPU.  Prints one JSON check line (not the metric)."""
    K = args.loopback
    name = "C5" if args.scene == "C5" else f"MW{K}"
    s = scenes.scene(name)
    fl = s["fluid"]
    bodies, verts = scenes.to_bodies(s["bodies"])
    cfg = lpe.default_fluid_config()
    wc = lpe.WorldConfig(1.0 / 120.0, 1.0, 1.0, 1.0)
    nt = args.warmup + args.steps

    one = lpe.Context(device)
    try:
        one.rigid_set_config(lpe.rigid_config(universe=s["U"]))
        one.rigid_upload(bodies, verts)
        one.sph_set_config(cfg)
        one.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        one.world_set_coupling(None)
        one.world_tick(1.0 / 120.0, args.prep + args.warmup)
        one.sync()
        t0 = time.perf_counter()
        one.world_tick(1.0 / 120.0, args.steps)
        one.sync()
        single = args.steps / (time.perf_counter() - t0)
        gpu_single = kernel_ms_per_tick([one], lambda n: one.world_tick(1.0 / 120.0, n))
    finally:
        one.close()

    edges = slab.slab_edges(fl["x"], K, cfg)
    ctxs = [lpe.Context(device) for _ in range(K)]
    try:
        for r, c in enumerate(ctxs):
            c.rigid_set_config(lpe.rigid_config(universe=s["U"]))
            c.rigid_upload(bodies, verts)
            slab.setup_rank(c, r, K, fl, edges, cfg, rebalance=args.rebalance)
            c.world_set_coupling(None)
        lpe.mg_loopback_run(ctxs, args.prep + args.warmup, world=wc)
        t0 = time.perf_counter()
        cpu0 = time.process_time()
        lpe.mg_loopback_run(ctxs, args.steps, world=wc)
        el = time.perf_counter() - t0
        host_cpu = time.process_time() - cpu0
        gpu_loop = kernel_ms_per_tick(ctxs, lambda n: lpe.mg_loopback_run(ctxs, n, world=wc))
        st = [c.sph_stats() for c in ctxs]
        info = [c.sph_slab_info() for c in ctxs]
        parts = [c.sph_download_owned() for c in ctxs]
        merged = slab.merge_owned(parts, len(fl["x"]))
        rb = [c.rigid_download() for c in ctxs]
        same = all(np.array_equal(rb[0][k], r[k]) for r in rb[1:] for k in ("x", "y", "angle"))
    finally:
        for c in ctxs:
            c.close()
    loop = args.steps / el
    print(json.dumps({"check": "loopback", "ranks": K, "scene": name, "particles": len(fl["x"]),
                      "prep_ticks": args.prep, "ticks_timed": args.steps,
                      "single_domain_ticks_per_s": round(single, 2),
                      "loopback_ticks_per_s_all_ranks_on_one_gpu": round(loop, 2),
                      "wall_ratio_loopback_over_single": round(single / loop, 3),
                      "owned": [x["slabOwned"] for x in st], "slots": [x["slabSlots"] for x in st],
                      "ghosts_in_max": [x["ghostsIn"] for x in st], "wire_records": st[0]["haloWire"][1],
                      "edges_columns": [int(e) for e in info[0]["edges"][1:-1]],
                      "finite": bool(np.isfinite(merged["x"]).all() and np.isfinite(merged["vy"]).all()),
                      "rigid_replicas_identical": bool(same), "max_cell_occupancy_rank0": st[0]["maxCellOccupancy"],
                      "gpu_kernel_ms_per_tick": {"single": gpu_single, "loopback_all_ranks": gpu_loop,
                                                 "ratio": round(gpu_loop / gpu_single, 3) if gpu_single else None},
                      "host_cpu_s_per_tick_loopback": round(host_cpu / args.steps, 5),
                      "note": "K ranks share one GPU: the ratio is the decomposition's overhead, not scaling; "
                              "gpu_kernel_ms_per_tick sums every launch's HIP-event time (all ranks) over "
                              "5 further ticks: the GPU work of the decomposition against the single domain's, "
                              "apart from the host's launch and rendezvous costs of K ranks in one process"}))


def kernel_ms_per_tick(ctxs, run, n=5):
    """Sum of the kernels' HIP-event times per tick over n ticks (every context)."""
    for c in ctxs:
        c.timing(True)
        c.timing_reset()
    run(n)
    for c in ctxs:
        c.sync()
    tot = 0.0
    for c in ctxs:
        tot += sum(ms for ms, _ in c.timing_read().values())
        c.timing(False)
    return round(tot / n, 3)


def rigid_microbench(lpe, device, reps=10):
    """One RigidBodyCollisionSystem::update (broadphase, narrowphase,
    colouring, PGS 10 it, position solver 10 it) on the metric scene's settled
    pile, the committed fixture tests/golden/pile_M_t250.npz, re-uploaded
    before every repetition: the same ~10k pairs / ~30k contacts every run, so
    the rigid kernels can be compared across runs (the live pile of the tick
    bench drifts with float-atomic summation order).  `jacobi`: the same with
    the opt-in Jacobi contact solver (pgsMode = LPE_PGS_JACOBI, 10 iterations)."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "pile_M_t250.npz"))
    names = ("k_bg_key", "k_bg_pairs", "k_narrow", "k_pair_colour", "k_pgs_colour", "k_pos_colour",
             "k_stripe_pairs", "k_stripe_setup", "k_group_colour", "k_stripe_layout", "k_stripe_fill",
             "k_pgs_stripes", "k_pos_stripes", "k_pgs_jacobi")

    def run(mode):
        ctx = lpe.Context(device)
        try:
            ctx.rigid_set_config(lpe.rigid_config(universe=32.0, pgsMode=mode))
            ctx.rigid_upload(z["bodies"], z["verts"])
            st = ctx.rigid_step()                       # warm
            ctx.timing(1)
            ctx.timing_reset()
            for _ in range(reps):
                ctx.rigid_upload(z["bodies"], z["verts"])
                ctx.rigid_step(stats=False)
            t = ctx.timing_read()
            ctx.timing(0)
        finally:
            ctx.close()
        us = {k: round(v[0] / max(v[1], 1) * 1e3, 1) for k, v in t.items()}
        step = sum(v[0] for v in t.values()) / reps * 1e3
        return st, round(step, 1), {k: us[k] for k in names if k in us}

    st, step, kus = run(lpe.PGS_GAUSS_SEIDEL)
    _, jstep, jus = run(lpe.PGS_JACOBI)
    return dict(fixture="tests/golden/pile_M_t250.npz", pairs=st["pairs"], contacts=st["contacts"],
                colours=st["pgsLevels"], colour_rounds=st["colourRounds"], reps=reps, step_kernels_us=step,
                kernels_us=kus, jacobi=dict(step_kernels_us=jstep, kernels_us=jus))


def bh_bench(lpe, scenes, device, reps=5):
    """BarnesHutSystem::update (barnes_hut.cpp:50-99) on the device (SURVEY.md
    §8(f) rank 4): the 20k-body Keplerian disk and the 65k-body clustered
    scene of tests/test_bh_gpu.py (parity-checked there, bit-exact fp64 against
    the restatement), one step = tree build + force walk + velocity update of
    every body.  bodies/s over the step's wall time (lpe_bh_step blocks until
    done) and per-stage device time (HIP events on the library's stream)."""
    out = {}
    for kind, n in (("disk", 20000), ("clustered", 65536)):
        s = scenes.bh_disk(n) if kind == "disk" else scenes.bh_clustered(n)
        cfg = lpe.bh_config(s["U"], softener=s["softener"])
        ctx = lpe.Context(device)
        try:
            ctx.bh_upload(s["x"], s["y"], s["vx"], s["vy"], s["m"])
            st = ctx.bh_step(cfg, 0.75)                 # warm
            ctx.sync()
            t0 = time.perf_counter()
            for _ in range(reps):
                ctx.bh_upload(s["x"], s["y"], s["vx"], s["vy"], s["m"])
                ctx.bh_step(cfg, 0.75)
            wall = (time.perf_counter() - t0) / reps
            ctx.timing(1)
            ctx.timing_reset()
            for _ in range(reps):
                ctx.bh_upload(s["x"], s["y"], s["vx"], s["vy"], s["m"])
                ctx.bh_step(cfg, 0.75)
            t = ctx.timing_read()
            ctx.timing(0)
        finally:
            ctx.close()
        dev_us = sum(v[0] for v in t.values()) / reps * 1e3
        out[f"{kind}{n}"] = dict(bodies=n, nodes=st["nodes"], depth=st["depth"],
                                 bodies_per_s=round(n / wall, 1), step_ms_wall=round(wall * 1e3, 3),
                                 step_us_device=round(dev_us, 1),
                                 kernels_us={k: round(v[0] / reps * 1e3, 1) for k, v in sorted(t.items())},
                                 note="wall includes the upload and the per-level host read-back of the build")
    return out


def timed_windows(ctx, dt_tick, rate_hint, nwin=5, min_s=2.0, min_ticks=50):
    """>= nwin windows of >= min_s each, back to back."""
    per = max(min_ticks, int(rate_hint * min_s) + 1)
    rates = []
    for _ in range(nwin):
        ctx.sync()
        t0 = time.perf_counter()
        ctx.world_tick(dt_tick, per)
        ctx.sync()
        rates.append(per / (time.perf_counter() - t0))
    return dict(median=round(float(np.median(rates)), 2), rates=[round(r, 2) for r in rates],
                ticks_per_window=per, windows=nwin)


def one_tick_calls(ctx, dt_tick, n):
    """The drop-in path: one lpe_world_tick call per ECSSimulator::tick (the
    host mirror's IntegratorSystems, host/src/systems/integrators.cpp)."""
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(n):
        ctx.world_tick(dt_tick, 1)
    ctx.sync()
    return n / (time.perf_counter() - t0)


def strict_mode(ctx, dt_tick, fl, n=10):
    """Strict mode: the ECS is synchronised every tick -- the fluid and the
    bodies go host -> device before the tick and device -> host after it
    (fluid.cpp:250-302 gather, :496-524 write-back), as the reference's
    FluidSystem does every tick.  PCIe-inclusive; not the headline."""
    out = ctx.sph_download()
    bodies = ctx.rigid_download()
    verts = ctx._rkeep[1]
    mass = np.asarray(fl["mass"], np.float32)
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(n):
        ctx.sph_upload(out["x"], out["y"], out["vx"], out["vy"], mass, out["density"], out["pressure"])
        ctx.rigid_upload(bodies, verts)
        ctx.world_tick(dt_tick, 1)
        out = ctx.sph_download()
        bodies = ctx.rigid_download()
    return n / (time.perf_counter() - t0)


def config_lines(lpe, scenes, device, dt_tick, with_ref):
    """Device tick rates at BASELINE.json's other configs,
    each after the scene is in motion, over a window of >= 2 s; the rigid
    configs beside the reference's own rigid path (oracle/_ref, compiled from
    /root/reference by oracle/Makefile.ref; its PGS is the restatement, the
    reference's needs NEON) on this host's single core, and BASELINE.md's
    anchors measured in the build container."""
    out = {}
    # C2 is the dam break (a transient by definition: timed right after the
    # dam opens); C4 is timed settled, 3,000 ticks in like scene M (VERDICT r4
    # item 4).  Both lead with the reference's own capped cells
    # (LPE_SPH_MODE_REF_CELL_CAP, the mode tests/test_configs_gpu.py pins at
    # these states); the unbounded rate is reported beside it.
    for name, prep in (("C2", 30), ("C4", 3000)):
        s = scenes.scene(name)
        fl = s["fluid"]
        b, v = scenes.to_bodies(s["bodies"])
        ctx = lpe.Context(device)
        try:
            ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
            ctx.rigid_upload(b, v)
            ctx.sph_set_config(lpe.default_fluid_config())
            ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
            ctx.world_set_coupling(None)
            ctx.world_tick(dt_tick, prep)
            ctx.sph_set_mode(lpe.SPH_MODE_REF_CELL_CAP)
            ctx.world_tick(dt_tick, 10)
            ctx.sph_diag(False)                       # restart the window totals
            w = timed_windows(ctx, dt_tick, 500.0, nwin=3, min_s=1.0)
            st = ctx.sph_stats()
            ctx.sph_set_mode(0)
            wu = timed_windows(ctx, dt_tick, 500.0, nwin=3, min_s=1.0)
        finally:
            ctx.close()
        over = st["overCapCellsTotal"]
        spread = (max(w["rates"]) - min(w["rates"])) / w["median"]
        out[name] = dict(desc=s["desc"], ticks_per_s=w["median"], windows=w, window_spread=round(spread, 4),
                         prep_ticks=prep, cells="the reference's 64-particle cells (LPE_SPH_MODE_REF_CELL_CAP)",
                         fluid_particles=len(fl["x"]), bodies=len(b), max_cell_occupancy=st["maxCellOccupancy"],
                         cells_over_64=st["overCapCells"],
                         reference_envelope=dict(max_cell_occupancy_window=st["maxCellOccupancyTotal"],
                                                 cells_over_64_window=over, inside=over == 0),
                         unbounded_cells_mode=dict(ticks_per_s=wu["median"], windows=wu))
    anchors = {"C1": (555.0, 600), "C3": (12.1, 240)}
    for name in ("C1", "C3"):
        s = scenes.rigid_scene(name)
        b, v = scenes.to_bodies(s["bodies"])
        cfg = lpe.rigid_config(universe=s["U"], pgs_iterations=s["pgs_iterations"])
        ctx = lpe.Context(device)
        try:
            ctx.rigid_set_config(cfg)
            ctx.rigid_upload(b, v)
            ctx.world_tick(dt_tick, 240 if name == "C3" else 60)       # the pile forms / the stack settles
            warm = ctx.rigid_download()
            w = timed_windows(ctx, dt_tick, 1000.0, nwin=3, min_s=1.0)
            pairs, contacts = ctx.rigid_contacts()
        finally:
            ctx.close()
        line = dict(desc=s["desc"], ticks_per_s=w["median"], windows=w, bodies=len(b), pgs_iterations=s["pgs_iterations"],
                    pairs=int(len(pairs)), contacts=int(len(contacts)),
                    reference_anchor=dict(ticks_per_s=anchors[name][0], where="BASELINE.md §2: the reference's own "
                                          "rigid path, -O2, 1 core of the build container's Xeon"))
        if with_ref:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle  # noqa: E402  (baseline only)
            if oracle.ref_available():
                nt = 1
                t0 = time.perf_counter()
                while True:                     # bounded sample: >= 1 s of the reference
                    oracle.ref_rigid_ticks(cfg, warm, v, nt, dt_tick)
                    el = time.perf_counter() - t0
                    if el > 1.0 or nt >= 512:
                        break
                    nt *= 2
                    t0 = time.perf_counter()
                line["reference_this_host"] = dict(ticks_per_s=round(nt / el, 2), ticks=nt, cores=1,
                                                   kind="reference", cpu_model=cpu_model())
            # the restatement's rigid tick on the same state (oracle/rigid_oracle.cpp, 1 thread): the
            # calibration of cpu_baseline's "port" against the reference
            bb, nt, t0 = warm, 0, time.perf_counter()
            while True:
                bb, _ = oracle.rigid_tick(cfg, bb, v, dt_tick)
                nt += 1
                el = time.perf_counter() - t0
                if el > 1.0 or nt >= 512:
                    break
            line["restatement_this_host"] = dict(ticks_per_s=round(nt / el, 2), ticks=nt, cores=1, kind="port",
                                                 cpu_model=cpu_model())
            if "reference_this_host" in line:
                line["restatement_over_reference"] = round(line["restatement_this_host"]["ticks_per_s"]
                                                           / line["reference_this_host"]["ticks_per_s"], 3)
        out[name] = line
    return out


def launch_ranks(n, cmd=None):
    """`python bench.py --gpus N` without a launcher: start N rank processes
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets
    them, rendezvous on 127.0.0.1) from this parent, which never touches the
    GPU, and return the first non-zero status of the children (0 if none).
    cmd: the rank command (default: this script with the same arguments)."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def envelope_all_ranks(dist, st):
    """The reference-envelope counters of the timed window over every rank
    (ADVICE r4 / VERDICT r4 item 3): cells over the reference's 64 summed (a
    ghost column's cells are counted by both ranks that hold it, so the sum
    may count a cell twice; `inside` is exact), the largest occupancy the
    maximum."""
    over, occ = st["overCapCellsTotal"], st["maxCellOccupancyTotal"]
    if dist is not None:
        import torch
        t = torch.tensor([over], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        m = torch.tensor([occ], dtype=torch.int64)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        over, occ = int(t.item()), int(m.item())
    return dict(max_cell_occupancy_window=occ, cells_over_64_window=over, inside=over == 0)


def slab_leg(lpe, scenes, slab, dist, rank, world, device, scene_name, prep, warmup, steps, transport,
             rebalance, keep=False, cells="ref"):
    """One sharded run: scene `scene_name`'s fluid in `world` x-slabs (one per
    rank), the rigid pass replicated, `prep` + `warmup`
    untimed ticks, then exactly `steps` ticks bracketed by barriers and device
    syncs; elapsed = the maximum over ranks.  cells="ref" (as the 1-GPU
    line): after the prep every rank switches to the reference's 64-particle
    cells (LPE_SPH_MODE_REF_CELL_CAP with the global count; the ranks then
    file at least 3 ghost columns, tests/test_slab_gpu.py::
    test_slab_capped_cells_bit_exact); the all-rank envelope says how many
    cells exceeded 64 in the window.  transport: "rccl" (the product path) or
    "gloo" (host-staged, lpe_mg_init_host: two ranks may share one GPU;
    rehearsal only).  Returns a dict; with keep the context stays open
    (leg["ctx"])."""
    s = scenes.scene(scene_name)
    fl = s["fluid"]
    bodies, verts = scenes.to_bodies(s["bodies"])
    cfg = lpe.default_fluid_config()
    ctx = lpe.Context(device)
    ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
    ctx.rigid_upload(bodies, verts)
    edges = slab.slab_edges(fl["x"], world, cfg)
    wire = slab.wire_capacity(fl["x"], edges, cfg, band=slab.BAND_CAP_WIRE if cells == "ref" else slab.BAND)
    slab.setup_rank(ctx, rank, world, fl, edges, cfg, rebalance=rebalance, wire_cap=wire)
    if transport == "gloo":
        ctx.mg_init_host(world, rank, slab.GlooTransport(rank, world))
    else:
        uid = slab.broadcast_uid(lpe.mg_unique_id() if rank == 0 else None, rank)
        ctx.mg_init_rccl(world, rank, uid)
    ctx.world_set_coupling(None)
    dt_tick = 1.0 / 120.0
    ctx.world_tick(dt_tick, prep)
    if cells == "ref":                    # (every rank, at the same tick: the ghost band follows the mode)
        ctx.sph_set_global_count(len(fl["x"]))
        ctx.sph_set_mode(lpe.SPH_MODE_REF_CELL_CAP)
    ctx.world_tick(dt_tick, warmup)
    ctx.sync()
    ctx.sph_diag(False)
    dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    ctx.world_tick(dt_tick, steps)
    ctx.sync()
    t1 = time.perf_counter()
    dist.barrier()
    import torch
    mine_s = t1 - t0
    st = ctx.sph_stats()
    mine = dict(rank=rank, ms_per_tick=mine_s / steps * 1e3, owned=st["slabOwned"], slots=st["slabSlots"],
                ghosts_in=st["ghostsIn"], wire=st["haloWire"],
                comm_ranks=ctx.mg_info()["comm_ranks"] if transport == "rccl" else world,
                edges=[int(e) for e in ctx.sph_slab_info()["edges"][1:-1]])
    every = [None] * world
    dist.all_gather_object(every, mine)
    t = torch.tensor([mine_s], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    env = envelope_all_ranks(dist, st)
    slow = max(every, key=lambda e: e["ms_per_tick"])
    n = len(fl["x"])
    leg = dict(scene=scene_name, desc=s["desc"], fluid_particles=n, rigid_bodies=len(bodies), prep_ticks=prep,
               ticks_timed=steps, elapsed=elapsed, ticks_per_s=round(steps / elapsed, 2),
               particle_ticks_per_s=round(n * steps / elapsed, 1),
               particle_substeps_per_s=round(10 * n * steps / elapsed, 1),
               ranks=dict(ranks_seen=every[0]["comm_ranks"], world_size=world, transport=transport,
                          ms_per_tick=[round(e["ms_per_tick"], 4) for e in every],
                          slowest_rank=slow["rank"], slowest_ms_per_tick=round(slow["ms_per_tick"], 4),
                          owned=[e["owned"] for e in every], slots=[e["slots"] for e in every],
                          ghosts_in_max=[e["ghosts_in"] for e in every], wire_records=every[0]["wire"],
                          edges_columns=every[0]["edges"]),
               reference_envelope=env,
               cells=("the reference's 64-particle cells (LPE_SPH_MODE_REF_CELL_CAP)" if cells == "ref"
                      else "unbounded cells"),
               reference_semantics=cells == "ref" or env["inside"])
    if keep:
        leg["ctx"] = ctx
        leg["fluid"] = fl
        leg["U"] = s["U"]
    else:
        ctx.close()
    return leg


def single_leg(lpe, scenes, device, scene_name, prep, warmup, steps, cells="ref"):
    """The same scene as ONE domain on this rank's GPU, in the slab ranks'
    cell semantics: the scaling baseline measured in the same run (ADVICE r4:
    a ticks/s ratio must not mix the capped and unbounded modes)."""
    s = scenes.scene(scene_name)
    fl = s["fluid"]
    bodies, verts = scenes.to_bodies(s["bodies"])
    ctx = lpe.Context(device)
    try:
        ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
        ctx.rigid_upload(bodies, verts)
        ctx.sph_set_config(lpe.default_fluid_config())
        ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        ctx.world_set_coupling(None)
        ctx.world_tick(1.0 / 120.0, prep)
        if cells == "ref":
            ctx.sph_set_mode(lpe.SPH_MODE_REF_CELL_CAP)
        ctx.world_tick(1.0 / 120.0, warmup)
        ctx.sph_diag(False)
        ctx.sync()
        t0 = time.perf_counter()
        ctx.world_tick(1.0 / 120.0, steps)
        ctx.sync()
        el = time.perf_counter() - t0
        st = ctx.sph_stats()
    finally:
        ctx.close()
    return dict(scene=scene_name, fluid_particles=len(fl["x"]), prep_ticks=prep, ticks_timed=steps,
                ticks_per_s=round(steps / el, 2),
                cells="the reference's 64-particle cells (LPE_SPH_MODE_REF_CELL_CAP)" if cells == "ref" else "unbounded cells",
                reference_envelope=dict(max_cell_occupancy_window=st["maxCellOccupancyTotal"],
                                        cells_over_64_window=st["overCapCellsTotal"],
                                        inside=st["overCapCellsTotal"] == 0))


def scaling_blocks(world, primary, strong_leg, c5_one, m_one):
    """The N-rank line's scaling blocks from its legs (slab_leg / single_leg
    dicts): `scaling_strong_c5` -- C5 over the ranks against C5 as one domain
    on one GPU (speedup, efficiency = rate_N / (N x rate_1)); `scaling_weak`
    -- MW{N} (primary) against scene M as one domain (efficiency = rate_N /
    rate_1, each rank holding an M-sized slab).  primary is the leg `value`
    was timed on (MW{N}, or C5 itself under --scene C5, then strong_leg is
    None and m_one is None)."""
    out = {}
    strong = strong_leg if strong_leg is not None else primary
    sc = dict(scene="C5", desc="2,097,152 SPH particles (fixed) over the ranks' x-slabs",
              fluid_particles=strong["fluid_particles"], ranks=world, ticks_per_s=strong["ticks_per_s"],
              single_gpu=c5_one, speedup=round(strong["ticks_per_s"] / c5_one["ticks_per_s"], 3),
              efficiency=round(strong["ticks_per_s"] / (world * c5_one["ticks_per_s"]), 4),
              reference_envelope=strong["reference_envelope"],
              reference_semantics=bool(strong["reference_envelope"]["inside"] and
                                       c5_one["reference_envelope"]["inside"]),
              slowest_ms_per_tick=strong["ranks"]["slowest_ms_per_tick"], ranks_detail=strong["ranks"])
    out["scaling_strong_c5"] = sc
    if m_one is not None:
        mw = primary["ticks_per_s"]
        n = primary["fluid_particles"]
        out["scaling_weak"] = dict(
            scene=primary["scene"], desc=primary["desc"], fluid_particles=n, ranks=world,
            ticks_per_s=mw, particle_ticks_per_s=round(n * mw, 1), particle_substeps_per_s=round(10 * n * mw, 1),
            value_is=f"{world} x {primary['scene']} ticks/s: the whole job's throughput in ticks/s of the "
                     f"256k-particle metric scene (each rank advances one M-sized slab per tick)",
            single_gpu=m_one, efficiency=round(mw / m_one["ticks_per_s"], 4),
            reference_semantics=bool(primary["reference_envelope"]["inside"] and m_one["reference_envelope"]["inside"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--scene", default="M")
    ap.add_argument("--prep", type=int, default=None,
                    help="untimed ticks that settle the scene before warmup (the pile forms); "
                         "default 3000 for M, 240 for the fluid-only C5")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the >=2 s windows, one-tick calls, strict mode and the C1-C4 lines")
    ap.add_argument("--no-density-microbench", action="store_true")
    ap.add_argument("--replicas", action="store_true",
                    help="N > 1: independent copies of the scene instead of the slab-sharded MW{N}")
    ap.add_argument("--loopback", type=int, default=0,
                    help="validation only: K slab ranks of MW{K} in this process on one GPU "
                         "(in-process transport); prints a check line, not the metric")
    ap.add_argument("--rebalance", type=int, default=10,
                    help="N > 1: move the slab edges towards equal counts every this many ticks (0: fixed)")
    ap.add_argument("--transport", choices=("rccl", "gloo"), default="rccl",
                    help="N > 1: the slab exchange over RCCL (default, the product path) or the host-staged "
                         "gloo transport (lpe_mg_init_host; ranks may share one GPU: rehearsal only)")
    ap.add_argument("--strong-prep", type=int, default=240,
                    help="N > 1: untimed ticks of the C5 strong-scaling leg (and its single-GPU baseline)")
    ap.add_argument("--cells", choices=("ref", "unbounded"), default="ref",
                    help="ref (default): the timed window runs the reference's 64-particle cells "
                         "(LPE_SPH_MODE_REF_CELL_CAP, fluid.hpp:56); unbounded: no per-cell cap")
    args = ap.parse_args()
    if args.prep is None:
        args.prep = 240 if args.scene == "C5" else 3000

    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not args.loopback:
        sys.exit(launch_ranks(args.gpus))       # (the parent makes no HIP call)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus and not args.loopback:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a {world}-rank run "
              f"as {args.gpus} GPU(s)", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        dist.init_process_group("gloo")

    lpe = _load("lpe", os.path.join(PKG, "lpe.py"))
    scenes = _load("scenes", os.path.join(PKG, "scenes.py"))
    slab = _load("slab", os.path.join(PKG, "slab.py"))
    if args.transport == "gloo" and world > 1:
        # rehearsal: ranks may share the GPUs there are (RCCL would refuse)
        local = local % max(1, lpe.device_count())
    if args.loopback:
        return loopback_check(args, lpe, scenes, slab, local)
    sharded = world > 1 and not args.replicas
    scene_name = f"MW{world}" if sharded and args.scene == "M" else args.scene
    dt_tick = 1.0 / 120.0

    def barrier():
        if dist is not None:
            dist.barrier()

    ranks_info = None
    if sharded:
        # the sharded path: slab_leg times exactly K ticks between barriers and
        # reports the maximum over ranks and the all-rank envelope
        leg = slab_leg(lpe, scenes, slab, dist, rank, world, local, scene_name, args.prep, args.warmup,
                       args.steps, args.transport, args.rebalance, keep=True, cells=args.cells)
        ctx, fl, elapsed = leg["ctx"], leg["fluid"], leg["elapsed"]
        s = dict(desc=leg["desc"], U=leg["U"])
        n_bodies = leg["rigid_bodies"]
        capped = args.cells == "ref"
        wstats = ctx.sph_stats()
        wstats["overCapCellsTotal"] = leg["reference_envelope"]["cells_over_64_window"]
        wstats["maxCellOccupancyTotal"] = leg["reference_envelope"]["max_cell_occupancy_window"]
        ranks_info = leg["ranks"]
    else:
        s = scenes.scene(scene_name)
        fl = s["fluid"]
        bodies, verts = scenes.to_bodies(s["bodies"])
        n_bodies = len(bodies)
        ctx = lpe.Context(local)
        ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
        ctx.rigid_upload(bodies, verts)
        ctx.sph_set_config(lpe.default_fluid_config())
        ctx.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        ctx.world_set_coupling(None)      # every body, reverse insertion (gatherRigidBodies view order)

        # scene preparation: the pentagons fall into the pool and settle into a
        # pile (the steady state: ~10k pairs, ~35k contacts); BASELINE.md times
        # the reference's pile the same way, after 240 warm-up ticks
        ctx.world_tick(dt_tick, args.prep)
        # the timed window in the reference's own cell semantics (its 64-slot
        # cells: dropped inserts, cross-cell reads; fluid.hpp:56, metal:237-240,
        # :281-283) -- the mode tests/test_configs_gpu.py pins at this state
        capped = args.cells == "ref"
        if capped:
            ctx.sph_set_mode(lpe.SPH_MODE_REF_CELL_CAP)
        ctx.world_tick(dt_tick, args.warmup)
        ctx.sync()

        ctx.sph_diag(False)               # restart the window totals (cells over the reference's 64)
        barrier()
        ctx.sync()
        t0 = time.perf_counter()
        ctx.world_tick(dt_tick, args.steps)
        ctx.sync()
        t1 = time.perf_counter()
        barrier()
        elapsed = t1 - t0
        wstats = ctx.sph_stats()
        if dist is not None:              # replicas: the slowest replica's window
            import torch
            t = torch.tensor([elapsed], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
            env = envelope_all_ranks(dist, wstats)
            wstats["overCapCellsTotal"] = env["cells_over_64_window"]
            wstats["maxCellOccupancyTotal"] = env["max_cell_occupancy_window"]
    extras = {}
    if world == 1 and not args.no_extras:
        rate = args.steps / elapsed
        extras["windows"] = timed_windows(ctx, dt_tick, rate)
        n1 = max(50, int(rate * 2.0))
        r1 = one_tick_calls(ctx, dt_tick, n1)
        extras["one_tick_calls"] = dict(ticks_per_s=round(r1, 2), ticks=n1,
                                        vs_multi_tick=round(r1 / extras["windows"]["median"], 4),
                                        note="lpe_world_tick(ctx, wc, 1) in a loop: the drop-in path "
                                             "(one call per ECSSimulator::tick)")
        extras["strict"] = dict(ticks_per_s=round(strict_mode(ctx, dt_tick, fl), 2),
                                note="ECS sync every tick: fluid + bodies uploaded before and downloaded "
                                     "after each tick (PCIe-inclusive, fluid.cpp:250-302 / :496-524)")
    # per-kernel durations: start/stop events carried by every launch on the
    # library's stream (hipExtLaunchKernelGGL), over a second window of the
    # same length (the event bookkeeping adds host work per launch, so it is
    # kept out of the window `value` is measured on)
    ctx.timing(1)
    ctx.timing_reset()
    ctx.world_tick(dt_tick, args.steps)
    times = ctx.timing_read()
    ctx.timing(False)
    stats = ctx.sph_stats()
    pairs, contacts = ctx.rigid_contacts()
    _, ncolours = ctx.rigid_colours()
    # (both downloads also check the capacity / overflow flags)
    out = ctx.sph_download_owned() if sharded else ctx.sph_download()
    settled = dict(fluid=out, bodies=ctx.rigid_download())
    n_rank = len(out["x"])
    render = render_bench(ctx, s["U"]) if world == 1 and not args.no_density_microbench else None

    strong_leg = None
    if sharded:
        barrier()
        ctx.close()        # (every rank past its last collective on this communicator)
        ctx = None
        if scene_name != "C5":
            # north_star's scaling claim: the fixed 2M-particle C5 scene over
            # the same ranks (strong scaling), in the same line
            strong_leg = slab_leg(lpe, scenes, slab, dist, rank, world, local, "C5", args.strong_prep,
                                  args.warmup, args.steps, args.transport, args.rebalance, cells=args.cells)

    if rank != 0:
        if dist is not None:
            dist.barrier()
        if ctx is not None:
            ctx.close()    # RCCL communicator torn down by every rank after the last barrier
        return

    assert np.isfinite(out["x"]).all() and np.isfinite(out["vy"]).all()
    n = n_rank                      # particles rank 0 owns (the whole scene unless sharded)
    cells = stats["gridDimX"] * stats["gridDimY"]
    # the roofline kernel: the SPH kernel with the largest share of the tick
    # (the rigid solvers are latency-bound single-workgroup sweeps with no
    # byte model; they are reported in kernels_us)
    modeled = {k: v for k, v in times.items() if kernel_bytes(k, n, cells) is not None}
    dname, (dms, dcalls) = max(modeled.items(), key=lambda kv: kv[1][0])
    overall = max(times.items(), key=lambda kv: kv[1][0])[0]
    avg_s = dms / max(dcalls, 1) / 1e3
    b = kernel_bytes(dname, n, cells)
    roof = None
    if b is not None:
        ach = b / avg_s / 1e9
        traffic, tsrc, tsame = pmc_traffic(dname) if world == 1 and args.scene == "M" else (None, None, False)
        roof = dict(kernel=dname, bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS,
                    unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4), traffic=traffic,
                    avg_us=round(avg_s * 1e6, 2), algorithmic_bytes=b)
        if tsrc:
            roof["traffic_source"] = tsrc + " (HBM bytes per launch, rocprofv3 PMC FETCH_SIZE x2 + WRITE_SIZE, " \
                                            "settled metric scene)"
            roof["traffic_same_build"] = tsame
            roof["traffic_frac_of_algorithmic"] = round(traffic / b, 3)
        ru, rsrc, rsame = rocprof_window(dname) if world == 1 and args.scene == "M" else (None, None, False)
        if ru:
            # the same kernel by rocprofv3's kernel trace (the profile committed
            # under profiles/): the tracer's own clock, beside the HIP events
            roof["rocprof"] = dict(avg_us=ru, achieved=round(b / (ru * 1e-6) / 1e9, 1),
                                   frac=round(b / (ru * 1e-6) / 1e9 / HBM_PEAK_GBS, 4), source=rsrc,
                                   same_build=rsame)
        vi, vsrc, vsame = pmc_valu(dname) if world == 1 and args.scene == "M" else (None, None, False)
        if vi:
            # the compute side of the same launch: VALU instructions (PMC) over
            # the live duration, against the chip's VALU issue rate
            roof["valu"] = dict(wave_insts=vi, achieved_ginst_s=round(vi / avg_s / 1e9, 1),
                                peak_ginst_s=VALU_PEAK_GINST, frac=round(vi / avg_s / 1e9 / VALU_PEAK_GINST, 4),
                                source=vsrc, same_build=vsame)
    # the whole tick against HBM: the staged
    # compulsory model B_tick = substeps x (152 B x N + 24 B x C) at the
    # measured tick rate
    btick = 10.0 * (152.0 * n + 24.0 * cells)
    tick_rate = args.steps / elapsed
    roof_tick = dict(model="10 x (152 B x N + 24 B x C) per tick (SURVEY.md §8(d))", bytes_per_tick=btick,
                     achieved=round(btick * tick_rate / 1e9, 1), unit="GB/s",
                     frac=round(btick * tick_rate / 1e9 / HBM_PEAK_GBS, 4), ticks_per_s=round(tick_rate, 2))
    dens = times.get("k_density")
    roof_d = None
    if dens:
        avg_d = dens[0] / max(dens[1], 1) / 1e3
        bd = kernel_bytes("k_density", n, cells)
        roof_d = dict(kernel="k_density", achieved=round(bd / avg_d / 1e9, 1), unit="GB/s",
                      frac=round(bd / avg_d / 1e9 / HBM_PEAK_GBS, 4), avg_us=round(avg_d * 1e6, 2))
    # weak scaling: every rank advances one M-sized SPH slab (sharded) or one
    # copy of the scene (replicas) per tick; strong scaling (C5, SURVEY.md
    # §8(d)): the one fixed 2M-particle scene, split over the ranks
    strong = args.scene == "C5" and not args.replicas
    value = (1 if strong else world) * args.steps / elapsed
    line = {
        "metric": "physics steps/sec at 256k SPH + 4k rigids; 1/2/4/8 MI355X vs HBM roofline",
        "value": round(value, 2),
        "unit": "ticks/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f32 (SPH), f64+f32 (rigid: fp64 geometry, fp32 PGS as the reference)",
        "data": "synthetic (seeded scene generator, SURVEY.md §8(d))",
        "config": {"workload": s["desc"] + f", ticks {args.prep + args.warmup}.."
                               f"{args.prep + args.warmup + args.steps} (settled pile)",
                   "scene": scene_name, "fluid_particles": len(fl["x"]),
                   "fluid_particles_rank0": n, "prep_ticks": args.prep,
                   "rigid_bodies": n_bodies, "substeps": 10, "dt": dt_tick,
                   "systems": ["FluidSystem (SPH + coupling)", "Boundary", "Gravity",
                               "RigidBodyCollision (broadphase, GJK/EPA, PGS 10 it, position 10 it)",
                               "Rotation", "Movement", "Sleep"],
                   "mode": "resident (ECS sync skipped inside the timed region)",
                   "cells": ("the reference's 64-particle cells (LPE_SPH_MODE_REF_CELL_CAP)" if capped
                             else "unbounded cells"),
                   "parallelism": (f"SPH x-slabs x{world} ({'RCCL' if args.transport == 'rccl' else 'gloo host-staged'}"
                                   f" halo + bbox/accumulator all-reduce), rigid pass replicated") if sharded else
                                  ("single GPU" if world == 1 else f"replica x{world}")},
        "roofline": roof,
        "roofline_density": roof_d,
        "roofline_tick": roof_tick,
        "kernels_us": {k: round(v[0] / max(v[1], 1) * 1e3, 2) for k, v in times.items()},
        "dominant_kernel": overall,
        "max_cell_occupancy": stats["maxCellOccupancy"],
        "reference_envelope": {
            "max_cell_occupancy_window": wstats["maxCellOccupancyTotal"],
            "cells_over_64_window": wstats["overCapCellsTotal"],
            "inside": wstats["overCapCellsTotal"] == 0,
            "note": "reference cells (2h) holding more than GPU_MAX_PER_CELL = 64 particles, summed over the "
                    "sub-steps of the timed window: where non-zero the reference drops inserts and reads "
                    "across cells (fluid.hpp:56, fluid_kernels.metal:237-240, :281-283); the window runs "
                    "LPE_SPH_MODE_REF_CELL_CAP (config.cells), which reproduces that behaviour exactly "
                    "(tests/test_configs_gpu.py checks both modes at this scene)"},
        "rigid": {"pairs": int(len(pairs)), "contacts": int(len(contacts)), "colours": int(ncolours)},
        "hw_queues": lpe.hw_queues(),
    }
    if ranks_info is not None:
        line["ranks"] = ranks_info
    if sharded:
        # the scaling baselines, measured in this run on rank 0's GPU while the
        # other ranks wait: each scene as ONE domain in the slab ranks' cell
        # semantics (args.cells: the reference's capped cells by default, as
        # the driver's own N=1 line), so every ratio compares one computation
        # 
        primary = dict(scene=scene_name, desc=s["desc"], fluid_particles=len(fl["x"]),
                       ticks_per_s=round(args.steps / elapsed, 2), reference_envelope=line["reference_envelope"],
                       ranks=ranks_info)
        c5_one = single_leg(lpe, scenes, local, "C5", args.strong_prep, args.warmup, args.steps, cells=args.cells)
        m_one = (single_leg(lpe, scenes, local, "M", args.prep, args.warmup, args.steps, cells=args.cells)
                 if scene_name != "C5" else None)
        line.update(scaling_blocks(world, primary, strong_leg, c5_one, m_one))
    line.update(extras)
    if world == 1 and not args.no_extras:
        # the same scene in the other cell mode
        ctx.sph_set_mode(0 if capped else lpe.SPH_MODE_REF_CELL_CAP)
        w = timed_windows(ctx, dt_tick, args.steps / elapsed, nwin=3, min_s=1.0)
        ctx.sph_set_mode(lpe.SPH_MODE_REF_CELL_CAP if capped else 0)
        line["unbounded_cells_mode" if capped else "ref_cell_cap_mode"] = dict(ticks_per_s=w["median"], windows=w)
        # the opt-in Jacobi contact solver on the same live scene (after the
        # timed windows: it changes the physics, not the reference's PGS)
        ctx.rigid_set_config(lpe.rigid_config(universe=s["U"], pgsMode=lpe.PGS_JACOBI))
        w = timed_windows(ctx, dt_tick, args.steps / elapsed, nwin=3, min_s=1.0)
        ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
        line["pgs_jacobi_mode"] = dict(ticks_per_s=w["median"], windows=w,
                                       note="opt-in Jacobi contact solver (pgsMode = LPE_PGS_JACOBI, 10 "
                                            "iterations), timed on the live scene after the windows above; "
                                            "not the reference's arithmetic (tests/test_jacobi_gpu.py)")
        line["configs"] = config_lines(lpe, scenes, local, dt_tick, not args.no_cpu_baseline)
    if world == 1 and not args.no_density_microbench:
        line["density_microbench"] = density_microbench(lpe, scenes, local)
        line["rigid_microbench"] = rigid_microbench(lpe, local)
        line["barnes_hut"] = bh_bench(lpe, scenes, local)
        line["render_density"] = render
    if world == 1 and not args.no_cpu_baseline and args.scene == "M":
        line["cpu_baseline"] = cpu_baseline(args.scene, settled)
    if world == 1 and args.scene == "M":
        line["dropin"] = dropin_record()
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()
    if ctx is not None:
        ctx.close()


if __name__ == "__main__":
    main()
