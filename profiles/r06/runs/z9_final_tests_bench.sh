# round 6 (z9, after z8 committed the same-build profiles): the final library -- the whole -m gpu suite, smoke, the default bench line (with the CPU baseline)
mkdir -p gpurun_out/r06g
export TMPDIR=/tmp
sha256sum little-physics-engine_amd/liblpe_hip.so > gpurun_out/r06g/lib_sha256.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r06g/pytest_gpu.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r06g/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06g/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u bench.py > gpurun_out/r06g/bench_line.json 2> gpurun_out/r06g/bench.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
exit 0
