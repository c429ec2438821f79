# round 4 (y): end-of-round evidence, part 3 (the final library): the full -m gpu suite, smoke(), 8-rank loopback lines (MW8, C5), the slab path in separate processes, C1 / C2 / C3 probes
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r04y_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04y_smoke.log 2>&1 || exit 1
timeout -k 10 240 python -u bench.py --loopback 8 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04y_loop_mw8.json 2> gpurun_out/r04y_loop_mw8.err || exit 1
timeout -k 10 240 python -u bench.py --loopback 8 --scene C5 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04y_loop_c5.json 2> gpurun_out/r04y_loop_c5.err || exit 1
for m in single slab1 slab1_loopback; do
  timeout -k 10 150 python -u profiles/slab_probe.py --only $m --prep 3000 --ticks 300 > gpurun_out/r04y_slab_$m.json 2> gpurun_out/r04y_slab_$m.err || exit 1
done
for s in C1 C2; do timeout -k 10 150 python -u profiles/small_probe.py --scene $s > gpurun_out/r04y_small_$s.json 2> gpurun_out/r04y_small_$s.err || exit 1; done
timeout -k 10 150 python -u profiles/small_probe.py --scene C3 --ticks 200 > gpurun_out/r04y_small_C3.json 2> gpurun_out/r04y_small_C3.err || exit 1
