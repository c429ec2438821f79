# round 3 (aa): rigid-bin scan as a plain fused prefix (k_scan_blocks gone from the tick head), prelaunch stats merged
# by the first forces pass (k_merge_prestats gone): parity + settled rates
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_host_mirror.py tests/test_slab_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03aa_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03aa_snap.log 2>&1 || exit 1
for rep in 1 2 3; do
  TOPK=12 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03aa_rates.txt 2>&1 || exit 1
done
