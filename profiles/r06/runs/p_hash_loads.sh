#!/bin/bash
# The hash's latency chains: k_bucket_permute's record loads hoisted above the
# rank chain and k_scan_rows' bbox partials eight a thread in flight (default)
# against the previous library (profiles/_var/liblpe_prev.so), alternating.
set -e
mkdir -p gpurun_out/hl
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/hl/snap.log 2>&1
for rep in 1 2 3; do
  TOPK=14 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/new /' >> gpurun_out/hl/ab.txt 2>&1
  LPE_LIB=profiles/_var/liblpe_prev.so TOPK=14 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed 's/^/prev /' >> gpurun_out/hl/ab.txt 2>&1
done
cat gpurun_out/hl/ab.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sph_gpu.py tests/test_configs_gpu.py -k "not c5" > gpurun_out/hl/pytest.log 2>&1
tail -2 gpurun_out/hl/pytest.log
