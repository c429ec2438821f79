# round 6 (a): the off-grid fix and the lagged grid / slot growth -- the SPH and slab parity suites
mkdir -p gpurun_out/r06a
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_sph_gpu.py tests/test_slab_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r06a/pytest_sph_slab.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r06a/pytest_sph_slab.log
exit $rc
