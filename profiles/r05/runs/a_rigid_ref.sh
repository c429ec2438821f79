# round 5 (a): the rigid path against the reference's own fixtures at bench scale (rigid_pileM_t1, rigid_C3_t240)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rigid_gpu.py -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/r05a_rigid.log 2>&1; rc=$?; echo "pytest rc=$rc"; exit $rc
