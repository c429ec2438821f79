# round 5 (zl): the final library: the whole -m gpu suite, smoke, the default bench line, and rocprofv3 over the bench command
mkdir -p gpurun_out/r05zl
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05zl/pytest_gpu.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05zl/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/r05zl/bench_line.json 2> gpurun_out/r05zl/bench.err; rc=$?; echo "bench rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
exit 0
