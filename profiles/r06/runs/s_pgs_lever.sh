#!/bin/bash
# The rigid solvers' lever-arm perpendiculars staged once per solve (no negate +
# move per contact: 258 instructions in the step block instead of 272) against
# the previous library (profiles/_var/liblpe_prev.so), alternating from the
# settled snapshot; then the rigid / world / config parity tests.
set -e
mkdir -p gpurun_out/pl
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/pl/snap.log 2>&1
for rep in 1 2 3; do
  TOPK=6 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/lever /' >> gpurun_out/pl/ab.txt 2>&1
  LPE_LIB=profiles/_var/liblpe_prev.so TOPK=6 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/prev /' >> gpurun_out/pl/ab.txt 2>&1
done
cat gpurun_out/pl/ab.txt
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_rigid_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_jacobi_gpu.py -m gpu -k "not c5" > gpurun_out/pl/pytest.log 2>&1
tail -2 gpurun_out/pl/pytest.log
