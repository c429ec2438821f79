# round 4 (gg): one fork event for the prelaunch and the position solver, and no prelaunch join between the ticks of one call: parity; A/B against the evidence library (profiles/ab/liblpe_prev.so, sha256 f7d0a73a) on the settled scene M (snapshot, 600 ticks, alternating, 3 each) and C2 / C1
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_slab_gpu.py tests/test_rigid_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04gg_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r04gg_snap.log 2>&1 || exit 1
for r in 1 2 3; do
  LPE_LIB=profiles/ab/liblpe_prev.so timeout -k 10 100 python -u profiles/snapshot.py --load 600 >> gpurun_out/r04gg_M.txt 2>&1 || exit 1
  timeout -k 10 100 python -u profiles/snapshot.py --load 600 >> gpurun_out/r04gg_M.txt 2>&1 || exit 1
done
for s in C2 C1; do
  LPE_LIB=profiles/ab/liblpe_prev.so timeout -k 10 150 python -u profiles/small_probe.py --scene $s > gpurun_out/r04gg_prev_$s.json 2> gpurun_out/r04gg_prev_$s.err || exit 1
  timeout -k 10 150 python -u profiles/small_probe.py --scene $s > gpurun_out/r04gg_new_$s.json 2> gpurun_out/r04gg_new_$s.err || exit 1
done
