# round 4 (w): end-of-round evidence, part 2: same-build PMC passes (copied into profiles/r04 so the bench line reads them), the contract bench line, rocprofv3 kernel stats of the settled metric scene
mkdir -p gpurun_out
export TMPDIR=/tmp
bash profiles/pmc_collect.sh gpurun_out/r04w_pmc || exit 1
find gpurun_out/r04w_pmc -name "*.csv" -size +2M -delete
cp gpurun_out/r04w_pmc/pmc_traffic.json gpurun_out/r04w_pmc/pmc_valu.json gpurun_out/r04w_pmc/pmc_density_pair.json profiles/r04/ || exit 1
timeout -k 10 500 python -u bench.py > gpurun_out/r04w_bench.json 2> gpurun_out/r04w_bench.err || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r04w_snap.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d /tmp/r04w_stats -o snap -- python3 -u profiles/snapshot.py --load 50 > gpurun_out/r04w_prof.log 2>&1 || exit 1
db=$(ls /tmp/r04w_stats/*.db | head -1)
python3 profiles/rocpd_summary.py $db > gpurun_out/r04w_kernel_stats_settled_M.txt 2>&1 || exit 1
du -sh gpurun_out
