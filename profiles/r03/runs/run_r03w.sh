# round 3 (w): PMC passes of the shipped build (stamped with its sha256), the contract bench line, kernel stats of the bench
mkdir -p gpurun_out
export TMPDIR=/tmp
bash profiles/pmc_collect.sh gpurun_out/r03w_pmc || exit 1
find gpurun_out/r03w_pmc -name "*.csv" -size +2M -delete
timeout -k 10 400 python -u bench.py > gpurun_out/r03w_bench.json 2> gpurun_out/r03w_bench.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03w_stats -o bench -- python -u bench.py --steps 50 --no-extras > gpurun_out/r03w_stats.log 2>&1 || exit 1
find gpurun_out/r03w_stats -name "*kernel_trace.csv" -delete
du -sh gpurun_out
