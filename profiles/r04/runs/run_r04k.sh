# round 4 (k): slab path costs in separate processes (single / 1-rank RCCL / 1-rank loopback); prelaunch stream priority A/B; no-prelaunch A/B
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in single slab1 slab1_loopback; do
  timeout -k 10 200 python -u profiles/slab_probe.py --only $m --prep 3000 --ticks 300 > gpurun_out/r04k_slab_$m.json 2> gpurun_out/r04k_slab_$m.err || exit 1
done
timeout -k 10 300 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline > gpurun_out/r04k_bench_prio.json 2> gpurun_out/r04k_bench_prio.err || exit 1
LPE_PSIDE_PRIO=0 timeout -k 10 300 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline > gpurun_out/r04k_bench_noprio.json 2> gpurun_out/r04k_bench_noprio.err || exit 1
LPE_NO_PRELAUNCH=1 timeout -k 10 300 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline > gpurun_out/r04k_bench_nopre.json 2> gpurun_out/r04k_bench_nopre.err || exit 1
