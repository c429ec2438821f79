# round 3 (jj): end-of-session evidence after the rigid head trims (full -m gpu suite, stamped PMC, bench line, settled stats) + C1 host probe
# the contract bench line, rocprofv3 stats of the settled scene
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03jj_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
bash profiles/pmc_collect.sh gpurun_out/r03jj_pmc || exit 1
find gpurun_out/r03jj_pmc -name "*.csv" -size +2M -delete
timeout -k 10 400 python -u bench.py > gpurun_out/r03jj_bench.json 2> gpurun_out/r03jj_bench.err || exit 1
TOPK=40 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03jj_stats -o snap -- python -u profiles/snapshot.py --load 60 > gpurun_out/r03jj_prof.log 2>&1 || exit 1
find gpurun_out/r03jj_stats -name "*kernel_trace.csv" -delete
timeout -k 10 120 python -u profiles/host_probe_c1.py > gpurun_out/r03jj_c1host.txt 2>&1 || exit 1
du -sh gpurun_out
