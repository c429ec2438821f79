# round 4 (g): density tests, 1-rank slab with one HW queue per stream, C5 loopback, bench (8 and 4 HW queues), drop-in timing
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_sph_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r04g_pytest_sph.log 2>&1 || exit 1
timeout -k 10 300 python -u profiles/slab_probe.py --loop --timing > gpurun_out/r04g_slab1.json 2> gpurun_out/r04g_slab1.err || exit 1
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python -u profiles/slab_probe.py --loop > gpurun_out/r04g_slab1_q4.json 2> gpurun_out/r04g_slab1_q4.err || exit 1
timeout -k 10 300 python -u bench.py --loopback 8 --scene C5 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04g_loop_c5.json 2> gpurun_out/r04g_loop_c5.err || exit 1
timeout -k 10 500 python -u bench.py > gpurun_out/r04g_bench.json 2> gpurun_out/r04g_bench.err || exit 1
GPU_MAX_HW_QUEUES=4 timeout -k 10 500 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline > gpurun_out/r04g_bench_q4.json 2> gpurun_out/r04g_bench_q4.err || exit 1
timeout -k 10 600 python -u profiles/dropin_timing.py > gpurun_out/r04g_dropin.json 2> gpurun_out/r04g_dropin.err || exit 1
