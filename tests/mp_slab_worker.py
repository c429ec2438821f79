"""One slab rank of tests/test_slab_multiprocess.py, run as its own process.

    python tests/mp_slab_worker.py RANK WORLD PORT SCENE NTICKS OUT.npz

Joins a gloo process group (127.0.0.1:PORT), sets up slab RANK of the scene's
fluid on cuda:0 with the rigid pass replicated, installs the host-staged
transport (lpe_mg_init_host over slab.GlooTransport), runs NTICKS resident
world ticks (lpe_world_tick, one call per tick as the drop-in does) and
writes its owned particles, its bodies and the transport's call counts to
OUT.npz.  With SCENE ending in ":mismatch" rank 1 declares a wire capacity
different from rank 0's, so the first exchange's sizes disagree: both ranks
must fail with an error, not hang."""
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "little-physics-engine_amd")


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def main():
    rank, world, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    scene_arg, nticks, out = sys.argv[4], int(sys.argv[5]), sys.argv[6]
    scene_name, _, mode = scene_arg.partition(":")
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lpe = _load("lpe", os.path.join(PKG, "lpe.py"))
    scenes = _load("scenes", os.path.join(PKG, "scenes.py"))
    slab = _load("slab", os.path.join(PKG, "slab.py"))
    s = scenes.scene(scene_name)
    fl = s["fluid"]
    b, v = scenes.to_bodies(s["bodies"])
    cfg = lpe.default_fluid_config()
    edges = slab.slab_edges(fl["x"], world)
    cap = slab.wire_capacity(np.asarray(fl["x"], np.float32), edges, cfg)
    if mode == "mismatch" and rank == 1:
        cap += 64
    tr = slab.GlooTransport(rank, world)
    ctx = lpe.Context(0)
    err = ""
    try:
        ctx.rigid_set_config(lpe.rigid_config(universe=s["U"]))
        ctx.rigid_upload(b, v)
        slab.setup_rank(ctx, rank, world, fl, edges, cfg, wire_cap=cap)
        ctx.world_set_coupling(np.arange(len(b) - 1, -1, -1, dtype=np.int32))
        ctx.mg_init_host(world, rank, tr)
        try:
            for _ in range(nticks):
                ctx.world_tick(1.0 / 120.0, 1)
            own = ctx.sph_download_owned(cap=len(fl["x"]))
            bodies = ctx.rigid_download()
        except lpe.LpeError as e:
            err = f"{e} | transport: {tr.last_error}"
            own, bodies = {}, np.zeros(0)
    finally:
        ctx.close()
    np.savez(out, err=np.array(err), bodies=bodies, calls=np.array([tr.calls["halo"], tr.calls["allreduce_f32"],
                                                                    tr.calls["allreduce_i64"]]),
             **{f"own_{k}": v for k, v in own.items()})
    # no collective after a failure: the peer may be gone
    if not err:
        dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
