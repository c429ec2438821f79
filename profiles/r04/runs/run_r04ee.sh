# round 4 (ee): end-of-round evidence for the final library (after the rigid-only detection stream change): same-build PMC passes (copied into profiles/r04 so the bench line reads them), the contract bench line, rocprofv3 kernel stats of the settled scene and of the bench command over its timing window
mkdir -p gpurun_out
export TMPDIR=/tmp
bash profiles/pmc_collect.sh gpurun_out/r04ee_pmc || exit 1
find gpurun_out/r04ee_pmc -name "*.csv" -size +2M -delete
cp gpurun_out/r04ee_pmc/pmc_traffic.json gpurun_out/r04ee_pmc/pmc_valu.json gpurun_out/r04ee_pmc/pmc_density_pair.json profiles/r04/ || exit 1
timeout -k 10 500 python -u bench.py > gpurun_out/r04ee_bench.json 2> gpurun_out/r04ee_bench.err || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d /tmp/r04ee_stats -o snap -- python3 -u profiles/snapshot.py --load 50 > gpurun_out/r04ee_prof.log 2>&1 || exit 1
db=$(ls /tmp/r04ee_stats/*.db | head -1)
python3 profiles/rocpd_summary.py $db > gpurun_out/r04ee_kernel_stats_settled_M.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/r04ee_bprof -o bench -- python3 bench.py --no-extras --no-density-microbench --no-cpu-baseline --steps 50 > gpurun_out/r04ee_bench_under_rocprof.json 2> gpurun_out/r04ee_bprof.log || exit 1
db=$(ls /tmp/r04ee_bprof/*.db | head -1)
python3 profiles/rocpd_summary.py $db --window-kernel k_forces_couple --window 500 > gpurun_out/r04ee_kernel_stats_bench_window.txt 2>&1 || exit 1
du -sh gpurun_out
