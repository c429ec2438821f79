#!/bin/bash
# A tile's own forces block issues its plan fetch (global -> LDS) before its filing
# check instead of after it: pf (= the in-tree library) against base (1f85a73f),
# alternating from the settled snapshot; then the SPH / config / world / slab /
# host-mirror tests.
mkdir -p gpurun_out/pp; rm -f gpurun_out/pp/ab.txt
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/pp/snap.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in base pf; do
    LPE_LIB=profiles/_var/liblpe_$v.so TOPK=12 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed "s/^/$v /" >> gpurun_out/pp/ab.txt 2>&1 || exit 1
  done
done
cat gpurun_out/pp/ab.txt
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sph_gpu.py tests/test_configs_gpu.py tests/test_world_gpu.py tests/test_slab_gpu.py tests/test_host_mirror.py -m gpu > gpurun_out/pp/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/pp/pytest.log
exit $rc
