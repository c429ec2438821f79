# round 4 (i): parity of the forces LDS image + branch-free list ring + single-wave solver steps; bench; small configs; slab; drop-in
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py tests/test_rigid_gpu.py tests/test_configs_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04i_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u bench.py > gpurun_out/r04i_bench.json 2> gpurun_out/r04i_bench.err || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C1 > gpurun_out/r04i_small_c1.json 2> gpurun_out/r04i_small_c1.err || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C2 > gpurun_out/r04i_small_c2.json 2> gpurun_out/r04i_small_c2.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04i_prof_c1 -o c1 -- python3 profiles/small_probe.py --scene C1 --rounds 1 > gpurun_out/r04i_prof_c1.log 2>&1 || exit 1
timeout -k 10 300 python -u profiles/slab_probe.py --loop --timing > gpurun_out/r04i_slab1.json 2> gpurun_out/r04i_slab1.err || exit 1
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python -u profiles/slab_probe.py --loop > gpurun_out/r04i_slab1_q4.json 2> gpurun_out/r04i_slab1_q4.err || exit 1
timeout -k 10 300 python -u bench.py --loopback 8 --scene C5 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04i_loop_c5.json 2> gpurun_out/r04i_loop_c5.err || exit 1
timeout -k 10 600 python -u profiles/dropin_timing.py > gpurun_out/r04i_dropin.json 2> gpurun_out/r04i_dropin.err || exit 1
