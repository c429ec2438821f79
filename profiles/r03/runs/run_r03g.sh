# round 3 (g): overlapped coupling phases in k_forces_couple: parity, tick rate vs base, phase trace
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 400 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_slab_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03g_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03g_snap.log 2>&1 || exit 1
for v in profiles/_var/liblpe_base.so little-physics-engine_amd/liblpe_hip.so profiles/_var/liblpe_base.so little-physics-engine_amd/liblpe_hip.so; do
  LPE_LIB=$v TOPK=12 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03g_rates.txt 2>&1 || exit 1
done
LPE_LIB=profiles/_var/liblpe_ft.so timeout -k 10 60 python -u profiles/forces_phase_trace.py > gpurun_out/r03g_ftrace.txt 2>&1
