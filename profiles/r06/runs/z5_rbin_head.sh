#!/bin/bash
# The tick's rigid-bin head: the histogram counted by the gather (no
# k_rbin_count launch in world ticks) and no k_rbin_sort (the fill copies the
# AABBs; the forces pass sorts a particle's few hits).  rb = the working tree,
# against cpl (the committed library), alternating from the settled snapshot;
# then the SPH / config / world / slab / host-mirror parity tests on the
# in-tree library (= rb2).
mkdir -p gpurun_out/rb; rm -f gpurun_out/rb/ab.txt
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/rb/snap.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in cpl rbs rb2; do
    LPE_LIB=profiles/_var/liblpe_$v.so TOPK=8 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed "s/^/$v /" >> gpurun_out/rb/ab.txt 2>&1 || exit 1
  done
done
cat gpurun_out/rb/ab.txt
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sph_gpu.py tests/test_configs_gpu.py tests/test_world_gpu.py tests/test_slab_gpu.py tests/test_host_mirror.py -m gpu > gpurun_out/rb/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/rb/pytest.log
exit $rc
