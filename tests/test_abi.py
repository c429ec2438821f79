"""CPU tests of the C-ABI boundary: the in-tree HIP library loads, exports every
symbol include/lpe.h declares, and its structs match the header layout.
No compute call is made (there is no GPU in the build container)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT, lpe

HEADER = os.path.join(ROOT, "include", "lpe.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(lpe_\w+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    L = ctypes.CDLL(lpe.LIB_PATH)
    names = header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert set(header_functions()) == set(lpe.SIGNATURES)


def test_abi_version_and_no_device_status():
    L = lpe.lib()
    assert L.lpe_abi_version() == lpe.ABI_VERSION == 2
    if lpe.device_count() == 0:
        h = ctypes.c_void_p()
        assert L.lpe_create(0, ctypes.byref(h)) == 6   # LPE_ERR_NO_DEVICE
        with pytest.raises(lpe.LpeError):
            lpe.Context(0)


def test_struct_layout_matches_header(tmp_path):
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "lpe.h"\n'
                   'int main(){printf("%zu %zu %zu %zu\\n", sizeof(lpe_fluid_config),'
                   ' sizeof(lpe_gpu_rigid), sizeof(lpe_sph_stats),'
                   ' offsetof(lpe_gpu_rigid, accumTorque)); return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    a, b, c, d = map(int, subprocess.check_output([str(exe)]).split())
    assert a == ctypes.sizeof(lpe.FluidConfig)
    assert b == lpe.RIGID_DTYPE.itemsize == 200
    assert c == ctypes.sizeof(lpe.SphStats)
    assert d == lpe.RIGID_DTYPE.fields["accumTorque"][1]


def test_default_config_matches_reference_defaults():
    """FluidConfig defaults (include/systems/fluid/fluid.hpp:131-200)."""
    c = lpe.default_fluid_config()
    assert (c.gravity, c.restDensity, c.stiffness) == (pytest.approx(9.81), 0.5, 200.0)
    assert c.viscosity == pytest.approx(0.03)
    assert c.numSubSteps == 10 and c.threadsPerGroup == 256
    assert c.gridConfig.smoothingLength == pytest.approx(0.05)
    assert c.impulseSolver.fluidForceScale == 100.0
    assert c.impulseSolver.maxSafeVelocitySq == 80.0
    assert c.positionSolver.relaxFactor == pytest.approx(0.9)
