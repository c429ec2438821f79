# round 4 (p): forces in-wave helper lanes (A/B LPE_FORCES_NOHELP x2), colouring chunk prefetch: parity, probes, forces trace
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > gpurun_out/r04p_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C1 > gpurun_out/r04p_small_c1.json 2> gpurun_out/r04p_small_c1.err || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline > gpurun_out/r04p_bench_help$i.json 2> gpurun_out/r04p_bench_help$i.err || exit 1
  LPE_FORCES_NOHELP=1 timeout -k 10 300 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline > gpurun_out/r04p_bench_nohelp$i.json 2> gpurun_out/r04p_bench_nohelp$i.err || exit 1
done
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r04p_snap.log 2>&1 || exit 1
LPE_LIB=profiles/_var/liblpe_ft.so timeout -k 10 120 python -u profiles/forces_trace.py > gpurun_out/r04p_ftrace.txt 2>&1 || exit 1
