# round 3 (gg): scan + rank + permute in one launch (k_hash_fused), the cell stats in k_density: parity, A/B
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/m240.py > gpurun_out/r03gg_m240.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_host_mirror.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03gg_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03gg_snap.log 2>&1 || exit 1
for rep in 1 2; do
  echo "NO_HASH_FUSION" >> gpurun_out/r03gg_rates.txt
  LPE_NO_HASH_FUSION=1 TOPK=10 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03gg_rates.txt 2>&1 || exit 1
  echo "FUSED" >> gpurun_out/r03gg_rates.txt
  TOPK=10 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03gg_rates.txt 2>&1 || exit 1
done
