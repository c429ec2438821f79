# round 6 (g): GPU_MAX_HW_QUEUES 4 (the box's default) vs 8 (INTEGRATION.md's advice) on the default bench line, alternating
mkdir -p gpurun_out/r06g
export TMPDIR=/tmp
for i in 1 2; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --no-extras --no-density-microbench --no-cpu-baseline --steps 200 > gpurun_out/r06g/q${q}_$i.json 2> gpurun_out/r06g/q${q}_$i.err; rc=$?; [ $rc -eq 0 ] || exit $rc
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/r06g/q${q}_$i.json').read().strip().splitlines()[-1]); print('q$q run$i', d['value'], d['hw_queues'])"
  done
done
