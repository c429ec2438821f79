# round 4 (h): parity of the single-wave solver steps and the 8-B density stores, slab-path costs, bench (8 / 4 HW queues), drop-in timing
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_rigid_gpu.py tests/test_sph_gpu.py tests/test_world_gpu.py -q --timeout 180 --timeout-method thread > gpurun_out/r04h_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u bench.py > gpurun_out/r04h_bench.json 2> gpurun_out/r04h_bench.err || exit 1
timeout -k 10 300 python -u profiles/slab_probe.py --loop --timing > gpurun_out/r04h_slab1.json 2> gpurun_out/r04h_slab1.err || exit 1
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python -u profiles/slab_probe.py --loop > gpurun_out/r04h_slab1_q4.json 2> gpurun_out/r04h_slab1_q4.err || exit 1
GPU_MAX_HW_QUEUES=4 timeout -k 10 500 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline > gpurun_out/r04h_bench_q4.json 2> gpurun_out/r04h_bench_q4.err || exit 1
timeout -k 10 300 python -u bench.py --loopback 8 --scene C5 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04h_loop_c5.json 2> gpurun_out/r04h_loop_c5.err || exit 1
timeout -k 10 600 python -u profiles/dropin_timing.py > gpurun_out/r04h_dropin.json 2> gpurun_out/r04h_dropin.err || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C1 > gpurun_out/r04h_small_c1.json 2> gpurun_out/r04h_small_c1.err || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C2 > gpurun_out/r04h_small_c2.json 2> gpurun_out/r04h_small_c2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04h_prof_c1 -o c1 -- python3 profiles/small_probe.py --scene C1 --rounds 1 > gpurun_out/r04h_prof_c1.log 2>&1 || exit 1
