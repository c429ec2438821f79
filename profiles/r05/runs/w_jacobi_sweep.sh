# round 5 (w): Jacobi kernel time vs iteration count; atomics vs plain stores (profiling variant)
mkdir -p gpurun_out/r05w
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
for it in 0 1 10 40; do
  ITERS=$it MODES=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05w_$it -o run -- python3 -u profiles/jacobi_ab.py > gpurun_out/r05w/it$it.log 2>&1; rc=$?; echo "it $it rc=$rc"; ok $rc
  cp $(find /tmp/r05w_$it -name '*kernel_stats.csv') gpurun_out/r05w/it${it}_stats.csv
done
ITERS=10 MODES=1 LPE_LIB=profiles/r05/var/liblpe_jplain.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05w_plain -o run -- python3 -u profiles/jacobi_ab.py > gpurun_out/r05w/plain.log 2>&1; rc=$?; echo "plain rc=$rc"; ok $rc
cp $(find /tmp/r05w_plain -name '*kernel_stats.csv') gpurun_out/r05w/plain_stats.csv
exit 0
