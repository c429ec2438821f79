"""CPU tests of the slab decomposition's host logic (little-physics-engine_amd/
slab.py): equal-count edges, ownership, buffer sizing, the owned-set merge,
and the torch.distributed plumbing on a world_size-2 gloo group."""
import importlib.util
import os
import socket
import sys

import numpy as np
import pytest

from conftest import PKG, scenes

_spec = importlib.util.spec_from_file_location("slab", os.path.join(PKG, "slab.py"))
slab = importlib.util.module_from_spec(_spec)
sys.modules["slab"] = slab
_spec.loader.exec_module(slab)


def test_edges_equal_count_and_ownership():
    fl = scenes.scene("small96_0")["fluid"]
    x = np.float32(fl["x"])
    for n in (1, 2, 3, 8):
        e = slab.slab_edges(x, n)
        assert len(e) == n + 1 and np.isneginf(e[0]) and np.isposinf(e[-1])
        assert (np.diff(e) > 0).all()
        own = slab.owners(x, e)
        cnt = np.bincount(own, minlength=n)
        assert cnt.sum() == len(x)
        assert cnt.max() - cnt.min() <= max(2, len(x) // (10 * n))   # equal count, lattice ties aside
        for r in range(n):                                           # [x0, x1) per slab
            xs = x[own == r]
            assert (xs >= e[r]).all() and (xs < e[r + 1]).all()


def test_edge_value_goes_right():
    e = np.array([-np.inf, 1.0, np.inf], np.float32)
    assert list(slab.owners(np.float32([0.99999994, 1.0, 1.0000001]), e)) == [0, 1, 1]


def test_ghost_capacity_covers_strip():
    fl = scenes.scene("small96_0")["fluid"]
    x = np.float32(fl["x"])
    e = slab.slab_edges(x, 2)
    halo = 0.2
    strip = int(((x >= e[1] - halo) & (x < e[1] + halo)).sum())
    assert slab.ghost_capacity(x, e, halo, factor=1.0, floor=0) >= strip // 2
    assert slab.ghost_capacity(x, e, halo) >= 4 * (strip // 2)


def _parts(n, nr, rng):
    perm = rng.permutation(n)
    chunks = np.array_split(perm, nr)
    parts = []
    for c in chunks:
        p = {k: (c * 10 + j).astype(np.float32) for j, k in enumerate(slab.FIELDS)}
        p["id"] = c.astype(np.int32)
        parts.append(p)
    return parts


def test_merge_owned_roundtrip_and_errors():
    rng = np.random.default_rng(0)
    n = 1000
    parts = _parts(n, 3, rng)
    m = slab.merge_owned(parts, n)
    for j, k in enumerate(slab.FIELDS):
        np.testing.assert_array_equal(m[k], (np.arange(n) * 10 + j).astype(np.float32))
    lost = [dict(p) for p in parts]
    lost[1] = {k: v[1:] for k, v in lost[1].items()}
    with pytest.raises(ValueError, match="lost"):
        slab.merge_owned(lost, n)
    dup = parts + [{k: v[:1] for k, v in parts[0].items()}]
    with pytest.raises(ValueError, match="duplicated"):
        slab.merge_owned(dup, n)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        uid = bytes(range(128)) if rank == 0 else None
        got = slab.broadcast_uid(uid, rank)
        rng = np.random.default_rng(1)
        n = 500
        parts = _parts(n, world, rng)
        merged = slab.gather_owned(parts[rank], n, rank, world)
        if rank == 0:
            ok = all(np.array_equal(merged[k], (np.arange(n) * 10 + j).astype(np.float32))
                     for j, k in enumerate(slab.FIELDS))
            q.put(("r0", got == bytes(range(128)), ok))
        else:
            q.put(("r1", got == bytes(range(128)), merged is None))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_uid_and_gather():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = sorted(q.get(timeout=5) for _ in range(2))
    for p in procs:
        assert p.exitcode == 0
    assert res == [("r0", True, True), ("r1", True, True)]
