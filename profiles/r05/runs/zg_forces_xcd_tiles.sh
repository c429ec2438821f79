# round 5 (zg): the forces pass's own tile blocks in XCD-contiguous runs (the filed heavy blocks first) vs plain order: parity, kernel times, HBM traffic
mkdir -p gpurun_out/r05zg
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05zg/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zg/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
for v in new plain new plain; do
  if [ $v = plain ]; then export LPE_LIB=profiles/r05/var/liblpe_plaintiles.so; else unset LPE_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05zg_$v -o run -- python3 -u profiles/heavy_modes.py >> gpurun_out/r05zg/modes_$v.jsonl 2> gpurun_out/r05zg/$v.log; rc=$?; echo "$v rc=$rc"; ok $rc
  cp $(find /tmp/r05zg_$v -name '*kernel_stats.csv') gpurun_out/r05zg/${v}_kernel_stats.csv; rm -rf /tmp/r05zg_$v
  python3 -c "
import csv,sys
rows={r['Name'].split('(')[0]:r for r in csv.DictReader(open('gpurun_out/r05zg/${v}_kernel_stats.csv'))}
print('$v', {k: round(float(rows[k]['AverageNs'])/1e3,2) for k in rows if any(x in k for x in ('k_density<true>','k_forces_couple'))})" >> gpurun_out/r05zg/summary.txt
done
for v in new plain; do
  if [ $v = plain ]; then export LPE_LIB=profiles/r05/var/liblpe_plaintiles.so; else unset LPE_LIB; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r05zg/pmc_$v -o $c -- python -u profiles/snapshot.py --load 20 > gpurun_out/r05zg/pmc_${v}_$c.log 2>&1; rc=$?; echo "pmc $v $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python profiles/pmc_traffic.py gpurun_out/r05zg/pmc_$v/FETCH_SIZE_counter_collection.csv gpurun_out/r05zg/pmc_$v/WRITE_SIZE_counter_collection.csv gpurun_out/r05zg/pmc_traffic_$v.json --last 50 --lib little-physics-engine_amd/liblpe_hip.so > /dev/null || exit 1
  python3 -c "
import json; t=json.load(open('gpurun_out/r05zg/pmc_traffic_$v.json')); print('$v traffic', {k: t[k]['hbm_bytes'] for k in ('k_forces_couple','k_density')})" >> gpurun_out/r05zg/summary.txt
done
unset LPE_LIB
exit 0
