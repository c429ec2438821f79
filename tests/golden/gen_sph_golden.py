"""Generates the SPH regression vectors under tests/golden/ from the CPU
oracle (oracle/sph_oracle.c).

The reference SPH path is Metal-only and holds no golden vectors (SURVEY.md
§8c), so these fixtures are NOT reference outputs: they pin the oracle against
unintended change ("parity unpinned" by reference execution).  Inputs are the
seeded scenes of little-physics-engine_amd/scenes.py.

    python tests/golden/gen_sph_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from conftest import scenes  # noqa: E402
import oracle  # noqa: E402

CASES = ["small64_8", "small48_0"]


def main():
    for name in CASES:
        s = scenes.scene(name)
        p = scenes.particles_aos(s["fluid"])
        rig = scenes.gather_rigids(s["bodies"])
        out, rout, acc, st = oracle.fluid_tick(p, rig, 1.0 / 120.0)
        cells, g = oracle.cells(p)
        np.savez_compressed(os.path.join(HERE, f"sph_{name}.npz"), particles_in=p, rigids_in=rig,
                            particles_out=out, rigids_out=rout, accum=acc, cells_in=cells,
                            grid=np.array([g.gridMinX, g.gridMinY, g.gridDimX, g.gridDimY]),
                            max_occ=st.maxOcc)
        print(name, p.shape, int(st.maxOcc))


if __name__ == "__main__":
    main()
