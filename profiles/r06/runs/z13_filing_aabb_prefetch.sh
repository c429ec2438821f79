#!/bin/bash
# The density pass's tile filing: a particle's first four candidate AABBs loaded
# after the staging barrier (in flight during the walk) instead of after the walk:
# hbb (= the in-tree library) against base (1f85a73f), alternating from the settled
# snapshot; then the SPH / config / world / slab / host-mirror tests.
mkdir -p gpurun_out/hb; rm -f gpurun_out/hb/ab.txt
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/hb/snap.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in base hbb; do
    LPE_LIB=profiles/_var/liblpe_$v.so TOPK=12 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed "s/^/$v /" >> gpurun_out/hb/ab.txt 2>&1 || exit 1
  done
done
cat gpurun_out/hb/ab.txt
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sph_gpu.py tests/test_configs_gpu.py tests/test_world_gpu.py tests/test_slab_gpu.py tests/test_host_mirror.py -m gpu > gpurun_out/hb/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/hb/pytest.log
exit $rc
