# round 4 (n): fused rigid launches; one stripe for small scenes (<= 1024 contact pairs): parity; forces LDS image A/B (LPE_FORCES_NOIMG) x2 alternating; C1 / C2 probes
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > gpurun_out/r04n_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C1 > gpurun_out/r04n_small_c1.json 2> gpurun_out/r04n_small_c1.err || exit 1
timeout -k 10 200 python -u profiles/small_probe.py --scene C2 > gpurun_out/r04n_small_c2.json 2> gpurun_out/r04n_small_c2.err || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline > gpurun_out/r04n_bench_img$i.json 2> gpurun_out/r04n_bench_img$i.err || exit 1
  LPE_FORCES_NOIMG=1 timeout -k 10 300 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline > gpurun_out/r04n_bench_noimg$i.json 2> gpurun_out/r04n_bench_noimg$i.err || exit 1
done
for m in single slab1 slab1_loopback; do
  timeout -k 10 200 python -u profiles/slab_probe.py --only $m --prep 3000 --ticks 300 > gpurun_out/r04n_slab_$m.json 2> gpurun_out/r04n_slab_$m.err || exit 1
done
