# round 3 (a): -m gpu tests, the default bench, the settled-M snapshot, the forces phase trace
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ] && { echo "stop: rc=$rc"; exit $rc; }; return 0; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03a_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc
timeout -k 10 450 python -u bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03a_snap.log 2>&1 || exit 1
LPE_LIB=profiles/_var/liblpe_ft.so timeout -k 10 120 python -u profiles/forces_phase_trace.py > gpurun_out/r03a_ftrace.txt 2>&1 || exit 1
DIAG=1 timeout -k 10 120 python -u profiles/snapshot.py --load 200 >> gpurun_out/r03a_snap.log 2>&1
