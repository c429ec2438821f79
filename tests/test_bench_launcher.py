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
