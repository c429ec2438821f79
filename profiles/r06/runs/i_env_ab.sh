# round 6 (i): runtime knobs on the default bench line (one context): kernel arguments in device memory, scratch reclaim
mkdir -p gpurun_out/r06i
export TMPDIR=/tmp
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline --steps 200 > gpurun_out/r06i/$tag.json 2> gpurun_out/r06i/$tag.err; local rc=$?; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.loads(open('gpurun_out/r06i/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['value'], 'forces', d['kernels_us'].get('k_forces_couple'), 'density', d['kernels_us'].get('k_density'), 'pgs', d['kernels_us'].get('k_pgs_stripes'))"; }
for i in 1 2; do
  run base_$i A=1
  run devkarg1_$i HIP_FORCE_DEV_KERNARG=1
  run devkarg0_$i HIP_FORCE_DEV_KERNARG=0
  run noreclaim_$i HSA_NO_SCRATCH_RECLAIM=1
done
