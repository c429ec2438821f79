# round 3 (cc): host enqueue time per world tick vs device time; scan_rows overflow-count load hoisted (rates)
mkdir -p gpurun_out
export TMPDIR=/tmp

timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03dd_snap.log 2>&1 || exit 1
timeout -k 10 120 python -u profiles/host_probe.py > gpurun_out/r03dd_host.txt 2>&1 || exit 1
for rep in; do
  TOPK=12 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03dd_rates.txt 2>&1 || exit 1
done
