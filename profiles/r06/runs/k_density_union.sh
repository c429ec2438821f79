#!/bin/bash
# Density: the wave-union walk (default) against the per-lane span walk
# (LPE_DENSITY_SPANS=1), alternating, from the settled snapshot; then the
# density / config parity tests.
set -e
mkdir -p gpurun_out/du
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/du/snap.log 2>&1
for rep in 1 2; do
  TOPK=6 timeout -k 10 60 python3 profiles/snapshot.py --load 1200 | sed 's/^/union /' >> gpurun_out/du/ab.txt 2>&1
  LPE_DENSITY_SPANS=1 TOPK=6 timeout -k 10 60 python3 profiles/snapshot.py --load 1200 | sed 's/^/spans /' >> gpurun_out/du/ab.txt 2>&1
done
cat gpurun_out/du/ab.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sph_gpu.py tests/test_configs_gpu.py -k "not c5" > gpurun_out/du/pytest.log 2>&1
tail -3 gpurun_out/du/pytest.log
