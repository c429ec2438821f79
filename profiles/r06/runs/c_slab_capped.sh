# round 6 (c): the reference's capped cells on slab ranks
mkdir -p gpurun_out/r06c
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_slab_gpu.py tests/test_configs_gpu.py -x -v --timeout 400 --timeout-method thread -k "capped or c5 or drift or world_tick_replicated or slab" > gpurun_out/r06c/pytest.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r06c/pytest.log
exit $rc
