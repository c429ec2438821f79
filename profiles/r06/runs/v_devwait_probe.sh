#!/bin/bash
# The device waits' concurrency probe: the serialised-dispatch world test, the
# world / rigid tests, then one PMC pass (counter collection serialises the
# dispatches: the tick must fall back to events, not spin into its watchdog).
set -e
mkdir -p gpurun_out/dp
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_world_gpu.py -m gpu > gpurun_out/dp/pytest.log 2>&1
tail -2 gpurun_out/dp/pytest.log
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/dp/snap.log 2>&1
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/dp/pmc -o M_fetch -- python -u profiles/snapshot.py --load 20 > gpurun_out/dp/pmc.log 2>&1
echo "pmc rc=$?"
tail -2 gpurun_out/dp/pmc.log
