"""The slab decomposition's exchange protocol across processes (SURVEY.md
§8(e)).

RCCL refuses two ranks on one GPU, so the 8-GPU bench is the only place the
RCCL transport meets a second rank.  These tests run the same protocol --
per sub-step one exchange (the ghost halo with the sizes both ends declare,
and the bbox records), per tick the rigid accumulator all-reduce -- between
separate processes through the host-staged transport
(lpe_mg_init_host, slab.GlooTransport over torch.distributed gloo):

- CPU: the transport's size handshake on a world_size-2 gloo group (matching
  sizes move the bytes; differing sizes fail on both ends, no hang).
- GPU: two worker processes (tests/mp_slab_worker.py), each a slab rank on
  cuda:0, run resident world ticks; the merged state is bit-identical to the
  single domain run in this process, and a rank that declares a different
  wire capacity makes both ranks fail loudly."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT, lpe, scenes

import importlib.util

_spec = importlib.util.spec_from_file_location("slab", os.path.join(PKG, "slab.py"))
slab = importlib.util.module_from_spec(_spec)
sys.modules["slab"] = slab
_spec.loader.exec_module(slab)

WORKER = os.path.join(ROOT, "tests", "mp_slab_worker.py")
DT = 1.0 / 120.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _handshake_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        tr = slab.GlooTransport(rank, world)
        res = []
        # matching sizes: rank r sends its bytes (value 10 r + side), receives the neighbour's
        n = 37
        sL = np.full(n, 10 * rank + 1, np.uint8) if rank > 0 else None
        sR = np.full(n, 10 * rank + 2, np.uint8) if rank < world - 1 else None
        rL = np.zeros(n, np.uint8) if rank > 0 else None
        rR = np.zeros(n, np.uint8) if rank < world - 1 else None
        tr.halo(sL, sR, rL, rR)
        res.append(bool((rL is None or (rL == 10 * (rank - 1) + 2).all())
                        and (rR is None or (rR == 10 * (rank + 1) + 1).all())))
        # differing sizes (rank 1 sends and expects 5 bytes more): both ends raise
        m = n + 5 * rank
        sL = np.zeros(m, np.uint8) if rank > 0 else None
        sR = np.zeros(m, np.uint8) if rank < world - 1 else None
        rL = np.zeros(m, np.uint8) if rank > 0 else None
        rR = np.zeros(m, np.uint8) if rank < world - 1 else None
        try:
            tr.halo(sL, sR, rL, rR)
            res.append(False)
        except RuntimeError as e:
            res.append("sizes differ" in str(e))
        # reductions: float min, int64 sum with two's-complement wrap
        f = np.array([rank, -rank, 5.0], np.float32)
        tr.allreduce_f32(f, 1)
        i = np.array([rank + 1, 2 ** 62 if rank == 0 else 2 ** 62], np.int64)
        tr.allreduce_i64(i)
        res.append(bool(np.array_equal(f, np.float32([0, -(world - 1), 5]))))
        res.append(int(i[0]) == world * (world + 1) // 2 and int(i[1]) == -(2 ** 63))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_gloo_transport_handshake_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_handshake_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = sorted(q.get(timeout=5) for _ in range(2))
    for p in procs:
        assert p.exitcode == 0
    assert res == [(0, [True, True, True, True]), (1, [True, True, True, True])]


def _run_workers(scene, nticks, tmp_path, world=2, timeout=240):
    port = _free_port()
    outs = [str(tmp_path / f"rank{r}.npz") for r in range(world)]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, "-u", WORKER, str(r), str(world), str(port), scene, str(nticks),
                               outs[r]], env=env) for r in range(world)]
    try:
        codes = [p.wait(timeout=timeout) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    assert codes == [0] * world, codes
    return [dict(np.load(o)) for o in outs]


@pytest.mark.gpu
def test_two_process_slab_world_ticks_bit_exact(tmp_path):
    """Two slab ranks in two processes (gloo host-staged transport), 4
    resident world ticks of the coupled small96_12 scene: fluid and bodies
    bit-identical to the single domain, the rigid replicas identical."""
    s = scenes.scene("small96_12")
    nt = 4
    b, v = scenes.to_bodies(s["bodies"])
    one = lpe.Context(0)
    try:
        one.rigid_set_config(lpe.rigid_config(universe=s["U"]))
        one.rigid_upload(b, v)
        fl = s["fluid"]
        one.sph_set_config(lpe.default_fluid_config())
        one.sph_upload(fl["x"], fl["y"], fl["vx"], fl["vy"], fl["mass"], fl["density"], fl["pressure"])
        one.world_set_coupling(np.arange(len(b) - 1, -1, -1, dtype=np.int32))
        one.world_tick(DT, nt)
        ref = one.sph_download()
        rb_ref = one.rigid_download()
    finally:
        one.close()
    res = _run_workers("small96_12", nt, tmp_path)
    for r in res:
        assert str(r["err"]) == "", str(r["err"])
        # per sub-step one exchange (the ghost halo and the bbox all-reduce);
        # per tick the accumulator all-reduce.  From the second tick on,
        # sub-step 0 is prelaunched at the end of the tick before, so the
        # last tick leaves one exchange done for the next: 10 nt + 1
        assert list(r["calls"]) == [nt * 10 + 1, nt * 10 + 1, nt], r["calls"]
    parts = [{k[4:]: r[k] for k in r if k.startswith("own_")} for r in res]
    got = slab.merge_owned(parts, len(fl["x"]))
    for k in slab.FIELDS:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
    for k in ("x", "y", "angle", "vx", "vy", "omega"):
        np.testing.assert_array_equal(res[0]["bodies"][k], res[1]["bodies"][k], err_msg=k)
        np.testing.assert_array_equal(res[0]["bodies"][k], rb_ref[k], err_msg=k)


@pytest.mark.gpu
def test_two_process_size_mismatch_fails_on_both_ranks(tmp_path):
    """Rank 1 declares a larger wire capacity: the first exchange's sizes
    disagree, and both processes return an error (RCCL would hang or
    truncate)."""
    res = _run_workers("small96_12:mismatch", 1, tmp_path)
    for r in res:
        assert "sizes differ" in str(r["err"]), str(r["err"])
