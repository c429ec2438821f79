# round 4 (l): single-pass coupling in the forces pass: parity, forces trace, bench; C5 loopback with GPU-work accounting
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_slab_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04l_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r04l_snap.log 2>&1 || exit 1
LPE_LIB=profiles/_var/liblpe_ft.so timeout -k 10 120 python -u profiles/forces_trace.py > gpurun_out/r04l_ftrace.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline > gpurun_out/r04l_bench.json 2> gpurun_out/r04l_bench.err || exit 1
timeout -k 10 300 python -u bench.py --loopback 8 --scene C5 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04l_loop_c5.json 2> gpurun_out/r04l_loop_c5.err || exit 1
timeout -k 10 300 python -u bench.py --loopback 2 --scene C5 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04l_loop2_c5.json 2> gpurun_out/r04l_loop2_c5.err || exit 1
