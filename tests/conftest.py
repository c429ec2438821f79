"""Shared test fixtures.

Markers: `gpu` tests need an MI355X (run with -m gpu on the GPU box); every
other test runs on the CPU here.
"""
import importlib.util
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "little-physics-engine_amd")
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


lpe = _load("lpe", os.path.join(PKG, "lpe.py"))
scenes = _load("scenes", os.path.join(PKG, "scenes.py"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle  # noqa: E402  (oracle/oracle.py)
    return oracle


@pytest.fixture(scope="session")
def gpu_ctx():
    if lpe.device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests must run on the MI355X box")
    ctx = lpe.Context(0)
    yield ctx
    ctx.close()
