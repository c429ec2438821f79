# round 4 (y): end-of-round evidence, part 3 (the final library): the full -m gpu suite, smoke(), the drop-in timed through the EnTT host harness
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04y_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04y_smoke.log 2>&1 || exit 1
timeout -k 10 600 python -u profiles/dropin_timing.py > gpurun_out/r04y_dropin.json 2> gpurun_out/r04y_dropin.err || exit 1
