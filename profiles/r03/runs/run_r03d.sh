# round 3 (d): parity of the SPH/world paths, A/B base vs current (M snapshot + small configs), forces trace
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 400 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03d_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03d_snap.log 2>&1 || exit 1
for lib in profiles/_var/liblpe_base.so little-physics-engine_amd/liblpe_hip.so profiles/_var/liblpe_base.so little-physics-engine_amd/liblpe_hip.so; do
  LPE_LIB=$lib timeout -k 10 180 python -u profiles/config_ab.py --m >> gpurun_out/r03d_ab.jsonl 2>>gpurun_out/r03d_ab.err; rc=$?; ok $rc
done
LPE_LIB=profiles/_var/liblpe_ft.so timeout -k 10 120 python -u profiles/forces_phase_trace.py > gpurun_out/r03d_ftrace.txt 2>&1
LPE_LIB=profiles/_var/liblpe_pt.so timeout -k 10 120 python -u profiles/stripe_trace.py > gpurun_out/r03d_strace.txt 2>&1
