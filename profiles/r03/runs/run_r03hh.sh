# round 3 (hh): the detection's memsets folded into k_rb_prep, the rigid scans' block pass folded into k_rscan_final, inContact zeroed by k_rb_prep:
# parity, C1/C2/C3 and settled M rates (A/B LPE_NO_RSCAN_FUSION=1 for the scans)
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_rigid_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_host_mirror.py tests/test_slab_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03hh_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03hh_snap.log 2>&1 || exit 1
for rep in 1 2; do
  echo "NO_RSCAN_FUSION" >> gpurun_out/r03hh_ab.txt
  LPE_NO_RSCAN_FUSION=1 timeout -k 10 180 python -u profiles/config_ab.py --m >> gpurun_out/r03hh_ab.txt 2>&1 || exit 1
  echo "RSCAN_FUSION" >> gpurun_out/r03hh_ab.txt
  timeout -k 10 180 python -u profiles/config_ab.py --m >> gpurun_out/r03hh_ab.txt 2>&1 || exit 1
done
