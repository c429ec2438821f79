# round 5 (v): opt-in Jacobi contact solver: parity vs restatement, invariants, kernel times, tick rates
mkdir -p gpurun_out/r05v
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 600 python -u -m pytest tests/test_jacobi_gpu.py tests/test_rigid_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05v/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05v_ab -o run -- python3 -u profiles/jacobi_ab.py > gpurun_out/r05v/ab.log 2>&1; rc=$?; echo "ab rc=$rc"; ok $rc
cp $(find /tmp/r05v_ab -name '*kernel_stats.csv') gpurun_out/r05v/ab_kernel_stats.csv
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05v/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
for rep in 1 2; do
  PGS_MODE=1 timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05v/modes.jsonl 2>> gpurun_out/r05v/err.log; rc=$?; ok $rc
  timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05v/modes.jsonl 2>> gpurun_out/r05v/err.log; rc=$?; ok $rc
done
exit 0
