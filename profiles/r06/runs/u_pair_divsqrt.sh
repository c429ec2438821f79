#!/bin/bash
# The pair term's correctly rounded divisions and square root without the
# general sequences' range handling (div_inrange / sqrt_inrange) against the
# previous library (profiles/_var/liblpe_prev.so), alternating from the
# settled snapshot; then the SPH / config / world parity tests.
set -e
mkdir -p gpurun_out/pd
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/pd/snap.log 2>&1
for rep in 1 2 3; do
  TOPK=8 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/short /' >> gpurun_out/pd/ab.txt 2>&1
  LPE_LIB=profiles/_var/liblpe_prev.so TOPK=8 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/prev /' >> gpurun_out/pd/ab.txt 2>&1
done
cat gpurun_out/pd/ab.txt
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sph_gpu.py tests/test_configs_gpu.py tests/test_world_gpu.py tests/test_slab_gpu.py -m gpu > gpurun_out/pd/pytest.log 2>&1
tail -2 gpurun_out/pd/pytest.log
