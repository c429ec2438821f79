# round 3 (t): forces-pass neighbour terms past LPE_FORCES_T by helper waves: parity, A/B (T=0 off) on the settled scene
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/m240.py > gpurun_out/r03t_m240.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_host_mirror.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03t_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03t_snap.log 2>&1 || exit 1
for rep in 1 2; do
  for t in 0 16 24 32; do
    echo "T=$t" >> gpurun_out/r03t_rates.txt
    LPE_FORCES_T=$t TOPK=6 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03t_rates.txt 2>&1 || exit 1
  done
done
