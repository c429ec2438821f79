#!/bin/bash
# k_bucket_permute: the bin bounds and its first eight filed ids in one round trip
# (perm); + the forces pass's filed blocks checking their class count instead of
# the tile flag (permf, = the in-tree library), against cpl, alternating from the
# settled snapshot; then the SPH / config / world / slab / host-mirror tests.
mkdir -p gpurun_out/pf; rm -f gpurun_out/pf/ab.txt
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/pf/snap.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in cpl perm permf; do
    LPE_LIB=profiles/_var/liblpe_$v.so TOPK=12 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed "s/^/$v /" >> gpurun_out/pf/ab.txt 2>&1 || exit 1
  done
done
cat gpurun_out/pf/ab.txt
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sph_gpu.py tests/test_configs_gpu.py tests/test_world_gpu.py tests/test_slab_gpu.py tests/test_host_mirror.py -m gpu > gpurun_out/pf/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/pf/pytest.log
exit $rc
