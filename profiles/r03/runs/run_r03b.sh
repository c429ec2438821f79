# round 3 (b): -m gpu tests, bench, settled snapshot, A/B of the small configs and M
# (base = HEAD before the lagged detection check), the forces phase trace
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03b_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc
timeout -k 10 450 python -u bench.py > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err; rc=$?; echo "bench rc=$rc"; ok $rc
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03b_snap.log 2>&1 || exit 1
for lib in profiles/_var/liblpe_base.so little-physics-engine_amd/liblpe_hip.so; do
  LPE_LIB=$lib timeout -k 10 180 python -u profiles/config_ab.py --m >> gpurun_out/r03b_ab.jsonl 2>>gpurun_out/r03b_ab.err; rc=$?; ok $rc
done
LPE_LIB=profiles/_var/liblpe_ft.so timeout -k 10 120 python -u profiles/forces_phase_trace.py > gpurun_out/r03b_ftrace.txt 2>&1
