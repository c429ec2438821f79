# round 4 (x): where the pile blocks' coupling phase goes: forces trace of the shipped arithmetic (ft), without the rigid accumulators' atomics (LPE_XP_NOXACC), without the impulse term (LPE_XP_NOIMP) -- timing-only variants -- and with the block's per-rigid LDS accumulators (ftla); parity of the LDS accumulators; bench
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r04x_snap.log 2>&1 || exit 1
for v in ft ftnx ftni ftla; do
  LPE_LIB=profiles/_var/liblpe_$v.so timeout -k 10 120 python -u profiles/forces_trace.py > gpurun_out/r04x_ftrace_$v.txt 2>&1 || exit 1
done
timeout -k 10 500 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_slab_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04x_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u bench.py --no-cpu-baseline > gpurun_out/r04x_bench.json 2> gpurun_out/r04x_bench.err || exit 1
