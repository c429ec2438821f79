# round 4 (t): end-of-round evidence, part 1: k_group_colour stage trace, the full -m gpu suite, smoke(), C1 / C2 / C3 probes
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
LPE_LIB=profiles/_var/liblpe_pt.so timeout -k 10 200 python -u profiles/colour_trace.py > gpurun_out/r04t_ctrace.txt 2>&1; rc=$?; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04t_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04t_smoke.log 2>&1 || exit 1
for s in C1 C2; do timeout -k 10 200 python -u profiles/small_probe.py --scene $s > gpurun_out/r04t_small_$s.json 2> gpurun_out/r04t_small_$s.err || exit 1; done
timeout -k 10 200 python -u profiles/small_probe.py --scene C3 --ticks 200 > gpurun_out/r04t_small_C3.json 2> gpurun_out/r04t_small_C3.err || exit 1
