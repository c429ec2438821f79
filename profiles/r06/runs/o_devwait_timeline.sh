# round 6 (o): after the device waits: this round's library at settled M: the default bench line, then rocprofv3 over the bench command (its per-kernel window) and a two-tick timeline
mkdir -p gpurun_out/r06o
export TMPDIR=/tmp

timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r06o_prof -o bench -- python3 bench.py --no-extras --no-density-microbench --no-cpu-baseline --steps 60 --warmup 10 > gpurun_out/r06o/bench_under_rocprof.json 2> gpurun_out/r06o/prof.log; rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
db=$(ls /tmp/r06o_prof/*.db | head -1)
python3 profiles/rocpd_summary.py $db --window-kernel k_forces_couple --window 500 --json gpurun_out/r06o/rocprof_window.json > gpurun_out/r06o/kernel_stats_bench_window.txt 2>&1 || exit 1
python3 profiles/rocpd_summary.py $db --window-kernel k_forces_couple --window 20 --timeline 150 > gpurun_out/r06o/timeline_2ticks.txt 2>&1 || exit 1
rm -rf /tmp/r06o_prof

timeout -k 10 200 ./profiles/r06/probe/gap_probe 400 > gpurun_out/r06o/gap_probe4.txt 2>&1
