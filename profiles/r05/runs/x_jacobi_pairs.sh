# round 5 (x): Jacobi solver by pairs with LDS-resident rows: parity vs restatement, iteration sweep, world rates
mkdir -p gpurun_out/r05x
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 600 python -u -m pytest tests/test_jacobi_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05x/tests.log 2>&1; rc=$?; echo "tests rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
for it in 0 1 10 40; do
  ITERS=$it MODES=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05x_$it -o run -- python3 -u profiles/jacobi_ab.py > gpurun_out/r05x/it$it.log 2>&1; rc=$?; echo "it $it rc=$rc"; ok $rc
  cp $(find /tmp/r05x_$it -name '*kernel_stats.csv') gpurun_out/r05x/it${it}_stats.csv
done
ITERS=10 MODES=1 LPE_LIB=profiles/r05/var/liblpe_jplain.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05x_plain -o run -- python3 -u profiles/jacobi_ab.py > gpurun_out/r05x/plain.log 2>&1; rc=$?; echo "plain rc=$rc"; ok $rc
cp $(find /tmp/r05x_plain -name '*kernel_stats.csv') gpurun_out/r05x/plain_stats.csv
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05x/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
PGS_MODE=1 timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05x/modes.jsonl 2>> gpurun_out/r05x/err.log; rc=$?; ok $rc
timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05x/modes.jsonl 2>> gpurun_out/r05x/err.log; rc=$?; ok $rc
exit 0
