#!/bin/bash
# The rigid solvers' single-wave step loop two steps a trip with the prefetch
# buffers taking turns (no copy of the next step's registers) against
# the previous library (profiles/_var/liblpe_prev.so), alternating from the
# settled snapshot; then the rigid / world / config parity tests.
set -e
mkdir -p gpurun_out/pp
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/pp/snap.log 2>&1
for rep in 1 2 3; do
  TOPK=6 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/pingpong /' >> gpurun_out/pp/ab.txt 2>&1
  LPE_LIB=profiles/_var/liblpe_prev.so TOPK=6 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/prev /' >> gpurun_out/pp/ab.txt 2>&1
done
cat gpurun_out/pp/ab.txt
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rigid_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_jacobi_gpu.py -m gpu -k "not c5" > gpurun_out/pp/pytest.log 2>&1
tail -2 gpurun_out/pp/pytest.log
