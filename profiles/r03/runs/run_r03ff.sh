# round 3 (ff): end-of-session evidence for the shipped build: the full -m gpu suite, PMC passes (stamped),
# the contract bench line, rocprofv3 stats of the settled scene
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03ff_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
bash profiles/pmc_collect.sh gpurun_out/r03ff_pmc || exit 1
find gpurun_out/r03ff_pmc -name "*.csv" -size +2M -delete
timeout -k 10 400 python -u bench.py > gpurun_out/r03ff_bench.json 2> gpurun_out/r03ff_bench.err || exit 1
TOPK=40 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03ff_stats -o snap -- python -u profiles/snapshot.py --load 60 > gpurun_out/r03ff_prof.log 2>&1 || exit 1
find gpurun_out/r03ff_stats -name "*kernel_trace.csv" -delete
du -sh gpurun_out
