# round 5 (t): per-kernel durations (rocprofv3 kernel trace) of the settled M ticks, tile scheduling on / off
mkdir -p gpurun_out/r05t
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05t_snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05t_on -o run -- python3 -u profiles/heavy_modes.py > gpurun_out/r05t/on.log 2>&1; rc=$?; echo "on rc=$rc"; ok $rc
LPE_NO_HEAVY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05t_off -o run -- python3 -u profiles/heavy_modes.py > gpurun_out/r05t/off.log 2>&1; rc=$?; echo "off rc=$rc"; ok $rc
cp $(find /tmp/r05t_on -name '*kernel_stats.csv') gpurun_out/r05t/on_kernel_stats.csv
cp $(find /tmp/r05t_off -name '*kernel_stats.csv') gpurun_out/r05t/off_kernel_stats.csv
exit 0
