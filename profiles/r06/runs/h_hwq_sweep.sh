# round 6 (h): GPU_MAX_HW_QUEUES 1..8 on the default bench line (one context)
mkdir -p gpurun_out/r06h
export TMPDIR=/tmp
for q in 2 3 4 5 6 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline --steps 200 > gpurun_out/r06h/q${q}.json 2> gpurun_out/r06h/q${q}.err; rc=$?; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06h/q${q}.json').read().strip().splitlines()[-1]); print('q$q', d['value'], d['kernels_us'].get('k_pgs_stripes'), d['kernels_us'].get('k_forces_couple'), d['kernels_us'].get('k_density'))"
done
