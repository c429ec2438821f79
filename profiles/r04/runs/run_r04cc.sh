# round 4 (cc): rigid-only worlds detect and colour on the context stream (no side-stream joins on the serial path); lagged counts stored by k_compact into the pinned slot (no copy launch): parity; C1 / C3 probes (A/B against the round-4 evidence library, profiles/ab/liblpe_prev.so, on the same box)
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_rigid_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_slab_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04dd_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for s in C1 C3; do
    t=500; [ $s = C3 ] && t=200
    timeout -k 10 150 python -u profiles/small_probe.py --scene $s --ticks $t > gpurun_out/r04dd_new_${s}_$r.json 2> gpurun_out/r04dd_new_${s}_$r.err || exit 1
    LPE_LIB=profiles/ab/liblpe_prev.so timeout -k 10 150 python -u profiles/small_probe.py --scene $s --ticks $t > gpurun_out/r04dd_prev_${s}_$r.json 2> gpurun_out/r04dd_prev_${s}_$r.err || exit 1
  done
done
