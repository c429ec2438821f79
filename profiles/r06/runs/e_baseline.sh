# round 6 (e): this round's library at settled M: the default bench line, then rocprofv3 over the bench command (its per-kernel window) and a two-tick timeline
mkdir -p gpurun_out/r06e
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --no-cpu-baseline > gpurun_out/r06e/bench_line.json 2> gpurun_out/r06e/bench.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r06e_prof -o bench -- python3 bench.py --no-extras --no-density-microbench --no-cpu-baseline --steps 50 > gpurun_out/r06e/bench_under_rocprof.json 2> gpurun_out/r06e/prof.log; rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
db=$(ls /tmp/r06e_prof/*.db | head -1)
python3 profiles/rocpd_summary.py $db --window-kernel k_forces_couple --window 500 --json gpurun_out/r06e/rocprof_window.json > gpurun_out/r06e/kernel_stats_bench_window.txt 2>&1 || exit 1
python3 profiles/rocpd_summary.py $db --window-kernel k_forces_couple --window 20 --timeline 190 > gpurun_out/r06e/timeline_2ticks.txt 2>&1 || exit 1
rm -rf /tmp/r06e_prof
exit 0
