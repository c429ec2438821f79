#!/bin/bash
# k_forces_couple code size / spills: cpl = the coupling constants from an LDS
# copy; cpl2 = + the rare over-PAIR_CAP path with one inlined pair (was four);
# cpl3 = + one inlined impulse term per pair (was one per shape).  Alternating
# from the settled snapshot against the previous library; then the SPH /
# config / world / slab parity tests on the in-tree library (= cpl3).
mkdir -p gpurun_out/yc
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/yc/snap.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in prev cpl cpl2 cpl3; do
    LPE_LIB=profiles/_var/liblpe_$v.so TOPK=6 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed "s/^/$v /" >> gpurun_out/yc/ab.txt 2>&1 || exit 1
  done
done
cat gpurun_out/yc/ab.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sph_gpu.py tests/test_configs_gpu.py tests/test_world_gpu.py tests/test_slab_gpu.py -m gpu > gpurun_out/yc/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/yc/pytest.log
exit $rc
