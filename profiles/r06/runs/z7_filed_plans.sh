#!/bin/bash
# The forces pass's filed blocks fetch their tile's staging plan by filing code
# (written there by the density pass) in flight with the list entry, instead of
# by tile after it: plan (= the in-tree library) against permf, alternating from
# the settled snapshot; then the SPH / config / world / slab / host-mirror tests.
mkdir -p gpurun_out/pl; rm -f gpurun_out/pl/ab.txt
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/pl/snap.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in permf plan; do
    LPE_LIB=profiles/_var/liblpe_$v.so TOPK=12 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed "s/^/$v /" >> gpurun_out/pl/ab.txt 2>&1 || exit 1
  done
done
cat gpurun_out/pl/ab.txt
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sph_gpu.py tests/test_configs_gpu.py tests/test_world_gpu.py tests/test_slab_gpu.py tests/test_host_mirror.py -m gpu > gpurun_out/pl/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/pl/pytest.log
exit $rc
