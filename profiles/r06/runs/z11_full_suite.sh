#!/bin/bash
# the whole -m gpu suite on the final library (131 tests: z9's 130 + the voided-prelaunch test)
mkdir -p gpurun_out/fs
sha256sum little-physics-engine_amd/liblpe_hip.so > gpurun_out/fs/lib_sha256.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/fs/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/fs/pytest_gpu.log
exit $rc
