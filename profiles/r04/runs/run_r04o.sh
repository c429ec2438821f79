# round 4 (o): register-resident colour masks for groups of <= 256 bodies: parity; C1 / C3 probes; bench; rocprofv3 kernel stats of the bench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_rigid_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04o_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C1 > gpurun_out/r04o_small_c1.json 2> gpurun_out/r04o_small_c1.err || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C3 --ticks 200 > gpurun_out/r04o_small_c3.json 2> gpurun_out/r04o_small_c3.err || exit 1
timeout -k 10 500 python -u bench.py --no-cpu-baseline > gpurun_out/r04o_bench.json 2> gpurun_out/r04o_bench.err || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r04o_prof -o bench -- python3 bench.py --no-extras --no-density-microbench --no-cpu-baseline --steps 50 > gpurun_out/r04o_prof_bench.log 2>&1 || exit 1
db=$(ls /tmp/r04o_prof/*.db | head -1)
python3 profiles/rocpd_summary.py $db > gpurun_out/r04o_prof_bench.txt 2>&1 || exit 1
ls /tmp/r04o_prof > gpurun_out/r04o_prof_files.txt
