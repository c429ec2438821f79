# round 5 (m): heavy tiles (halves, up to 192, only with >= 64 coupling rigids): parity, trace, rates
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 900 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_slab_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05m_parity.log 2>&1; rc=$?; echo "parity rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05m_snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
LPE_LIB=profiles/r05/var/liblpe_ft.so timeout -k 10 120 python -u profiles/forces_trace.py > gpurun_out/r05m_trace_heavy.txt 2>&1; rc=$?; ok $rc
for rep in 1 2; do
  timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05m_modes.jsonl 2>> gpurun_out/r05m_err.log; rc=$?; ok $rc
  LPE_NO_HEAVY=1 timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05m_modes.jsonl 2>> gpurun_out/r05m_err.log; rc=$?; ok $rc
done
timeout -k 10 200 python -u profiles/config_ab.py >> gpurun_out/r05m_config_ab.jsonl 2>> gpurun_out/r05m_err.log; rc=$?; ok $rc
LPE_LIB=profiles/r05/var/liblpe_base.so timeout -k 10 200 python -u profiles/config_ab.py >> gpurun_out/r05m_config_ab.jsonl 2>> gpurun_out/r05m_err.log; rc=$?; ok $rc
exit 0
