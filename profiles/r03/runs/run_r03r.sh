# round 3 (r): in-bin sort without the scatter pass (k_bucket_permute): parity, A/B against LPE_NO_BUCKET=1, kernel times
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/m240.py > gpurun_out/r03r_m240.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_host_mirror.py tests/test_rigid_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03r_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03r_snap.log 2>&1 || exit 1
for rep in 1 2; do
  echo "NO_BUCKET" >> gpurun_out/r03r_rates.txt
  LPE_NO_BUCKET=1 TOPK=40 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03r_rates.txt 2>&1 || exit 1
  echo "BUCKET" >> gpurun_out/r03r_rates.txt
  TOPK=40 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03r_rates.txt 2>&1 || exit 1
done
for v in little-physics-engine_amd/liblpe_hip.so profiles/_var/liblpe_nopipe.so little-physics-engine_amd/liblpe_hip.so profiles/_var/liblpe_nopipe.so; do
  LPE_LIB=$v timeout -k 10 120 python -u profiles/rigid_ab.py >> gpurun_out/r03r_ab.txt 2>&1 || exit 1
done
