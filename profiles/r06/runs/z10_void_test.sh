#!/bin/bash
# the mode-switch / voided-prelaunch regression test (with the config tests it shares its cached M@240 state with)
mkdir -p gpurun_out/vt
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_configs_gpu.py -m gpu -k "mode_switch or M-240" > gpurun_out/vt/pytest.log 2>&1; rc=$?
tail -8 gpurun_out/vt/pytest.log
exit $rc
