# round 4 (a): GPU suite + bench after the lagged-overflow containment, the stripe CU cap and the capped-mode cell list
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04a_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 500 python -u bench.py > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err; rc2=$?; echo "bench rc=$rc2"
exit $(( rc2 ))
