# round 5 (y): Jacobi with the device-side grid (blocks by the live contact count): tests, kernel time, world rates
mkdir -p gpurun_out/r05y
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 600 python -u -m pytest tests/test_jacobi_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05y/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05y/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
PGS_MODE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05y_w -o run -- python3 -u profiles/heavy_modes.py > gpurun_out/r05y/modes_jacobi_prof.log 2>&1; rc=$?; echo "prof rc=$rc"; ok $rc
cp $(find /tmp/r05y_w -name '*kernel_stats.csv') gpurun_out/r05y/world_jacobi_stats.csv
PGS_MODE=1 timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05y/modes.jsonl 2>> gpurun_out/r05y/err.log; rc=$?; ok $rc
timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05y/modes.jsonl 2>> gpurun_out/r05y/err.log; rc=$?; ok $rc
exit 0
