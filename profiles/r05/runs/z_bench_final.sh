# round 5 (z): the default bench line and rocprofv3 --kernel-trace --stats of the bench command (window: last 50 ticks)
mkdir -p gpurun_out/r05z
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 900 python -u bench.py > gpurun_out/r05z/bench_line.json 2> gpurun_out/r05z/bench.err; rc=$?; echo "bench rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r05z_prof -o bench -- python3 bench.py --no-extras --no-density-microbench --no-cpu-baseline --steps 50 > gpurun_out/r05z/bench_under_rocprof.json 2> gpurun_out/r05z/prof.log; rc=$?; echo "prof rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
db=$(ls /tmp/r05z_prof/*.db | head -1)
python3 profiles/rocpd_summary.py $db --window-kernel k_forces_couple --window 500 > gpurun_out/r05z/kernel_stats_bench_window.txt 2>&1 || exit 1
python3 profiles/rocpd_summary.py $db > gpurun_out/r05z/kernel_stats_bench_all.txt 2>&1 || exit 1
exit 0
