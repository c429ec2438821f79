# round 4 (c): slab-path cost on one GPU (1-rank slab vs single domain), rocprof of the 8-rank C5 loopback, the bench line
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u profiles/slab_probe.py --timing > gpurun_out/r04c_slab1.json 2> gpurun_out/r04c_slab1.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04c_prof_c5loop -o loop -- python3 -u bench.py --loopback 8 --scene C5 --prep 20 --warmup 2 --steps 10 > gpurun_out/r04c_c5loop_prof.log 2>&1 || exit 1
find gpurun_out/r04c_prof_c5loop -name "*kernel_trace.csv" -delete
timeout -k 10 500 python -u bench.py > gpurun_out/r04c_bench.json 2> gpurun_out/r04c_bench.err || exit 1
