#!/bin/bash
# Density at five tiles per CU (1472 staged records, boundaries read from the
# global cell table, 32 KB LDS) against the previous library (four tiles per
# CU, profiles/_var/liblpe_prev.so), alternating from the settled snapshot;
# then the SPH / config / world / slab parity tests.
set -e
mkdir -p gpurun_out/do
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/do/snap.log 2>&1
for rep in 1 2 3; do
  TOPK=8 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/occ5 /' >> gpurun_out/do/ab.txt 2>&1
  LPE_LIB=profiles/_var/liblpe_prev.so TOPK=8 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/prev /' >> gpurun_out/do/ab.txt 2>&1
done
cat gpurun_out/do/ab.txt
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sph_gpu.py tests/test_configs_gpu.py tests/test_world_gpu.py tests/test_slab_gpu.py -m gpu > gpurun_out/do/pytest.log 2>&1
tail -2 gpurun_out/do/pytest.log
