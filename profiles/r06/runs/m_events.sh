#!/bin/bash
# (1) gap probe: blocked barrier packets on other queues; (2) the tick's fork
# events carried by their kernels' launches (default) against recorded ones
# (LPE_EVENT_RECORDS=1), alternating from the settled snapshot; (3) world /
# rigid / config parity tests.
set -e
mkdir -p gpurun_out/ev
timeout -k 10 200 ./profiles/r06/probe/gap_probe 400 > gpurun_out/ev/gap_probe3.txt 2>&1
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/ev/snap.log 2>&1
for rep in 1 2 3; do
  TOPK=3 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/carried /' >> gpurun_out/ev/ab.txt 2>&1
  LPE_EVENT_RECORDS=1 TOPK=3 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/recorded /' >> gpurun_out/ev/ab.txt 2>&1
done
cat gpurun_out/ev/gap_probe3.txt gpurun_out/ev/ab.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_world_gpu.py tests/test_configs_gpu.py -k "not c5" > gpurun_out/ev/pytest.log 2>&1
tail -3 gpurun_out/ev/pytest.log
