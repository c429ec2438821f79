# round 4 (u): one-pass k_stripe_setup (stripe count from the partials, batched pair loads), k_group_colour list by wave ballots: parity; colour trace; C1 / C3 probes; bench
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_rigid_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_slab_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04u_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
LPE_LIB=profiles/_var/liblpe_pt.so timeout -k 10 200 python -u profiles/colour_trace.py > gpurun_out/r04u_ctrace.txt 2>&1; rc=$?; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C1 > gpurun_out/r04u_small_C1.json 2> gpurun_out/r04u_small_C1.err || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C3 --ticks 200 > gpurun_out/r04u_small_C3.json 2> gpurun_out/r04u_small_C3.err || exit 1
timeout -k 10 500 python -u bench.py --no-cpu-baseline > gpurun_out/r04u_bench.json 2> gpurun_out/r04u_bench.err || exit 1
