# round 4 (e): the 1-rank slab with one hardware queue per stream (GPU_MAX_HW_QUEUES=8 from lpe.py), and the bench line
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_sph_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r04e_pytest_sph.log 2>&1 || exit 1
timeout -k 10 300 python -u profiles/slab_probe.py --loop --timing > gpurun_out/r04e_slab1.json 2> gpurun_out/r04e_slab1.err || exit 1
GPU_MAX_HW_QUEUES=4 timeout -k 10 300 python -u profiles/slab_probe.py --loop > gpurun_out/r04e_slab1_q4.json 2> gpurun_out/r04e_slab1_q4.err || exit 1
timeout -k 10 300 python -u bench.py --loopback 8 --scene C5 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04e_loop_c5.json 2> gpurun_out/r04e_loop_c5.err || exit 1
timeout -k 10 500 python -u bench.py > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err || exit 1
GPU_MAX_HW_QUEUES=4 timeout -k 10 500 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline > gpurun_out/r04e_bench_q4.json 2> gpurun_out/r04e_bench_q4.err || exit 1
