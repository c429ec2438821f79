# round 4 (b): the per-sub-step-ownership slab path: slab/world/config GPU tests, then the 8-rank loopback checks
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_slab_gpu.py tests/test_slab_multiprocess.py -v --timeout 240 --timeout-method thread > gpurun_out/r04b_pytest_slab.log 2>&1; rc=$?; echo "pytest slab rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
[ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04b_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --loopback 8 --scene C5 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04b_loop_c5.json 2> gpurun_out/r04b_loop_c5.err; echo "loop c5 rc=$?"
timeout -k 10 300 python -u bench.py --loopback 8 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04b_loop_mw8.json 2> gpurun_out/r04b_loop_mw8.err; echo "loop mw8 rc=$?"
exit 0
