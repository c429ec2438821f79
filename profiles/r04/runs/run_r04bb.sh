# round 4 (bb): rocprofv3 --kernel-trace --stats of the bench command itself (final library), summarised over the bench's per-kernel timing window (the last 50 ticks = 500 k_forces_couple launches), beside the line that run printed
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r04bb_prof -o bench -- python3 bench.py --no-extras --no-density-microbench --no-cpu-baseline --steps 50 > gpurun_out/r04bb_bench_under_rocprof.json 2> gpurun_out/r04bb_prof.log || exit 1
db=$(ls /tmp/r04bb_prof/*.db | head -1)
python3 profiles/rocpd_summary.py $db --window-kernel k_forces_couple --window 500 > gpurun_out/r04bb_kernel_stats_bench_window.txt 2>&1 || exit 1
python3 profiles/rocpd_summary.py $db > gpurun_out/r04bb_kernel_stats_bench_all.txt 2>&1 || exit 1
