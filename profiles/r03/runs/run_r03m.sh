# round 3 (l): tick head: couple records in the gather, one-launch rigid bins: parity, A/B, timeline
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_slab_gpu.py tests/test_host_mirror.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03m_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03m_snap.log 2>&1 || exit 1
for rep in 1 2; do
  LPE_RBIN_MULTI=1 TOPK=4 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03m_rates.txt 2>&1 || exit 1
  TOPK=4 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03m_rates.txt 2>&1 || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03m_trace -o trace -- python -u profiles/snapshot.py --load 60 > gpurun_out/r03m_prof.log 2>&1
