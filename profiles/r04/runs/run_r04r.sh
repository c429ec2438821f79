# round 4 (r): group colouring chain with per-pair masks in lanes (32-pair chunks): parity; C1 / C3 probes; bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_rigid_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_slab_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04r_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C1 > gpurun_out/r04r_small_c1.json 2> gpurun_out/r04r_small_c1.err || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C3 --ticks 200 > gpurun_out/r04r_small_c3.json 2> gpurun_out/r04r_small_c3.err || exit 1
timeout -k 10 500 python -u bench.py --no-cpu-baseline > gpurun_out/r04r_bench.json 2> gpurun_out/r04r_bench.err || exit 1
