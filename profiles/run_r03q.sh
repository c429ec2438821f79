# round 3 (q): PMC passes of the shipped build (stamped), the contract bench line, kernel stats of the bench
mkdir -p gpurun_out
export TMPDIR=/tmp
bash profiles/pmc_collect.sh gpurun_out/r03q_pmc || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r03q_bench.json 2> gpurun_out/r03q_bench.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03q_stats -o bench -- python -u bench.py --steps 50 --no-extras > gpurun_out/r03q_stats.log 2>&1 || exit 1
LPE_LIB=profiles/_var/liblpe_pt.so timeout -k 10 120 python -u profiles/stripe_trace.py > gpurun_out/r03q_strace.txt 2>&1
