# round 4 (z): end-of-round evidence, part 4 (the final library): 8-rank loopback lines (MW8, C5), the slab path in separate processes, C1 / C2 / C3 probes
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --loopback 8 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04z_loop_mw8.json 2> gpurun_out/r04z_loop_mw8.err || exit 1
timeout -k 10 300 python -u bench.py --loopback 8 --scene C5 --prep 60 --warmup 5 --steps 20 > gpurun_out/r04z_loop_c5.json 2> gpurun_out/r04z_loop_c5.err || exit 1
for m in single slab1 slab1_loopback; do
  timeout -k 10 200 python -u profiles/slab_probe.py --only $m --prep 3000 --ticks 300 > gpurun_out/r04z_slab_$m.json 2> gpurun_out/r04z_slab_$m.err || exit 1
done
for s in C1 C2; do timeout -k 10 200 python -u profiles/small_probe.py --scene $s > gpurun_out/r04z_small_$s.json 2> gpurun_out/r04z_small_$s.err || exit 1; done
timeout -k 10 200 python -u profiles/small_probe.py --scene C3 --ticks 200 > gpurun_out/r04z_small_C3.json 2> gpurun_out/r04z_small_C3.err || exit 1
