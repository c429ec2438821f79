#!/bin/bash
# The tick's cross-stream waits as one-wave k_wait_flag kernels polling a word
# the boundary passes' last workgroup stores (default) against hipStreamWaitEvent
# on carried events (LPE_EVENT_WAITS=1), alternating from the settled snapshot;
# then the world / config / rigid / host-mirror parity tests.
set -e
mkdir -p gpurun_out/ev2

timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/ev2/snap.log 2>&1
for rep in 1 2 3; do
  TOPK=3 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/devwait /' >> gpurun_out/ev2/ab.txt 2>&1
  LPE_EVENT_WAITS=1 TOPK=3 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/events /' >> gpurun_out/ev2/ab.txt 2>&1
done
cat gpurun_out/ev2/ab.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_rigid_gpu.py tests/test_host_mirror.py -m gpu -k "not c5" > gpurun_out/ev2/pytest.log 2>&1
tail -3 gpurun_out/ev2/pytest.log
