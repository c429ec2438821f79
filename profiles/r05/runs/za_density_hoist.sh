# round 5 (za): the tile filing's candidate-range loads hoisted before the density walk: parity, kernel times (settled M)
mkdir -p gpurun_out/r05za
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05za/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05za/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05za_on -o run -- python3 -u profiles/heavy_modes.py > gpurun_out/r05za/on.log 2>&1; rc=$?; echo "on rc=$rc"; ok $rc
cp $(find /tmp/r05za_on -name '*kernel_stats.csv') gpurun_out/r05za/on_kernel_stats.csv
LPE_LIB=profiles/r05/var/liblpe_prehoist.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05za_pre -o run -- python3 -u profiles/heavy_modes.py > gpurun_out/r05za/pre.log 2>&1; rc=$?; echo "pre rc=$rc"; ok $rc
cp $(find /tmp/r05za_pre -name '*kernel_stats.csv') gpurun_out/r05za/pre_kernel_stats.csv
exit 0
