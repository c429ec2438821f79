# round 4 (ff): end-of-round evidence for the final library, part 2: the full -m gpu suite, smoke(), 8-rank loopback lines (MW8, C5), the slab path in separate processes, C1 / C2 / C3 probes, the drop-in through the EnTT host harness; C1 / C3 A/B against the round-4 evidence library (profiles/ab/liblpe_prev.so)
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04ff_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04ff_smoke.log 2>&1 || exit 1
for s in C1 C2; do timeout -k 10 150 python -u profiles/small_probe.py --scene $s > gpurun_out/r04ff_small_$s.json 2> gpurun_out/r04ff_small_$s.err || exit 1; done
timeout -k 10 150 python -u profiles/small_probe.py --scene C3 --ticks 200 > gpurun_out/r04ff_small_C3.json 2> gpurun_out/r04ff_small_C3.err || exit 1
timeout -k 10 240 python -u bench.py --loopback 8 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04ff_loop_mw8.json 2> gpurun_out/r04ff_loop_mw8.err || exit 1
timeout -k 10 240 python -u bench.py --loopback 8 --scene C5 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04ff_loop_c5.json 2> gpurun_out/r04ff_loop_c5.err || exit 1
timeout -k 10 400 python -u profiles/dropin_timing.py > gpurun_out/r04ff_dropin.json 2> gpurun_out/r04ff_dropin.err || exit 1
for s in C1 C3; do
  t=500; [ $s = C3 ] && t=200
  LPE_LIB=profiles/ab/liblpe_prev.so timeout -k 10 150 python -u profiles/small_probe.py --scene $s --ticks $t > gpurun_out/r04ff_prev_$s.json 2> gpurun_out/r04ff_prev_$s.err || exit 1
  timeout -k 10 150 python -u profiles/small_probe.py --scene $s --ticks $t > gpurun_out/r04ff_new_$s.json 2> gpurun_out/r04ff_new_$s.err || exit 1
done
