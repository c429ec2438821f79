"""CPU tests of bench.py's multi-GPU entry (`--gpus N` used to
be ignored): without WORLD_SIZE it starts N rank processes itself (the
parent makes no HIP call), with WORLD_SIZE it refuses a world size that
differs from --gpus."""
import importlib.util
import os
import subprocess
import sys

from conftest import ROOT

_spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
bench = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(bench)

PRINT_ENV = ("import os; print('RANK', os.environ['RANK'], os.environ['LOCAL_RANK'], os.environ['WORLD_SIZE'], "
             "os.environ['MASTER_ADDR'], os.environ['MASTER_PORT'], flush=True)")


def test_launcher_starts_n_ranks_with_the_torchrun_environment(capfd):
    assert bench.launch_ranks(3, [sys.executable, "-c", PRINT_ENV]) == 0
    lines = sorted(line.split() for line in capfd.readouterr().out.splitlines() if line.startswith("RANK"))
    assert [l[1:4] for l in lines] == [["0", "0", "3"], ["1", "1", "3"], ["2", "2", "3"]]
    assert {l[4] for l in lines} == {"127.0.0.1"} and len({l[5] for l in lines}) == 1


def test_launcher_reports_a_failing_rank():
    code = "import os, sys; sys.exit(5 if os.environ['RANK'] == '1' else 0)"
    assert bench.launch_ranks(2, [sys.executable, "-c", code]) == 5


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr


ENVELOPE_RANK = """
import importlib.util, json, os, sys
import torch.distributed as dist
spec = importlib.util.spec_from_file_location('b', os.path.join(%r, 'bench.py'))
b = importlib.util.module_from_spec(spec); spec.loader.exec_module(b)
dist.init_process_group('gloo')
r = dist.get_rank()
st = dict(overCapCellsTotal=[0, 7][r], maxCellOccupancyTotal=[41, 70][r])
env = b.envelope_all_ranks(dist, st)
quiet = b.envelope_all_ranks(dist, dict(overCapCellsTotal=0, maxCellOccupancyTotal=[12, 30][r]))
print('ENV', r, json.dumps([env, quiet]), flush=True)
dist.barrier()
dist.destroy_process_group()
"""


def test_envelope_is_reduced_over_ranks(capfd):
    """an N-rank line's reference envelope covers every
    rank (gloo world 2 under the bench's own launcher): cells over 64 summed,
    the largest occupancy the maximum, `inside` only when no rank saw an
    over-full cell -- and every rank sees the same result."""
    assert bench.launch_ranks(2, [sys.executable, "-c", ENVELOPE_RANK % ROOT]) == 0
    import json
    got = {}
    for line in capfd.readouterr().out.splitlines():
        if line.startswith("ENV"):
            _, r, js = line.split(" ", 2)
            got[int(r)] = json.loads(js)
    assert got[0] == got[1]
    env, quiet = got[0]
    assert env == dict(max_cell_occupancy_window=70, cells_over_64_window=7, inside=False)
    assert quiet == dict(max_cell_occupancy_window=30, cells_over_64_window=0, inside=True)


def _leg(scene, tps, n, inside=True, slow=1.0):
    return dict(scene=scene, desc=scene, fluid_particles=n, ticks_per_s=tps,
                reference_envelope=dict(max_cell_occupancy_window=40, cells_over_64_window=0 if inside else 3,
                                        inside=inside),
                ranks=dict(slowest_ms_per_tick=slow, world_size=8))


def test_scaling_blocks_shape():
    """The N-rank line's scaling blocks: the C5 strong
    figure with its single-GPU rate, speedup and efficiency rate_N / (N rate_1),
    and the weak MW{N} figure as its own ticks/s and particle-ticks/s with the
    efficiency against scene M on one GPU -- the semantics flag false as soon
    as one window left the reference envelope."""
    prim = _leg("MW8", 700.0, 8 * 262144)
    strong = _leg("C5", 1200.0, 2097152, inside=False)
    c5_one = dict(scene="C5", ticks_per_s=260.0, reference_envelope=dict(inside=True))
    m_one = dict(scene="M", ticks_per_s=790.0, reference_envelope=dict(inside=True))
    out = bench.scaling_blocks(8, prim, strong, c5_one, m_one)
    sc, wk = out["scaling_strong_c5"], out["scaling_weak"]
    assert sc["fluid_particles"] == 2097152 and sc["ticks_per_s"] == 1200.0
    assert sc["speedup"] == round(1200 / 260, 3) and sc["efficiency"] == round(1200 / (8 * 260), 4)
    assert sc["reference_semantics"] is False
    assert wk["ticks_per_s"] == 700.0 and wk["particle_ticks_per_s"] == round(8 * 262144 * 700.0, 1)
    assert wk["efficiency"] == round(700 / 790, 4) and wk["reference_semantics"] is True
    # --scene C5: the primary leg is the strong one, no weak block
    out = bench.scaling_blocks(4, _leg("C5", 900.0, 2097152), None, c5_one, None)
    assert set(out) == {"scaling_strong_c5"} and out["scaling_strong_c5"]["efficiency"] == round(900 / 1040, 4)
