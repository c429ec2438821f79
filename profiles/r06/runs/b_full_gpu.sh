# round 6 (b): the whole -m gpu suite after the off-grid fix, the ADVICE fixes and the ECSSimulator harness; smoke
mkdir -p gpurun_out/r06b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r06b/pytest_gpu.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/r06b/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06b/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; cat gpurun_out/r06b/smoke.log | tail -2
exit $rc
