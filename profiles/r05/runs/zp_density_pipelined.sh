# round 5 (zp): density trips software-pipelined (the next trip's records read before this trip's arithmetic): parity, kernel times
mkdir -p gpurun_out/r05zp
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py tests/test_sph_gpu.py tests/test_world_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05zp/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zp/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
for v in new prev new prev; do
  if [ $v = prev ]; then export LPE_LIB=profiles/r05/var/liblpe_prev.so; else unset LPE_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05zp_$v -o run -- python3 -u profiles/heavy_modes.py >> gpurun_out/r05zp/modes_$v.jsonl 2> gpurun_out/r05zp/$v.log; rc=$?; echo "$v rc=$rc"; ok $rc
  cp $(find /tmp/r05zp_$v -name '*kernel_stats.csv') gpurun_out/r05zp/${v}_kernel_stats.csv; rm -rf /tmp/r05zp_$v
  python3 -c "
import csv,sys
rows={r['Name'].split('(')[0]:r for r in csv.DictReader(open('gpurun_out/r05zp/${v}_kernel_stats.csv'))}
print('$v', {k: round(float(rows[k]['AverageNs'])/1e3,2) for k in rows if any(x in k for x in ('k_density<true>','k_forces_couple'))})" >> gpurun_out/r05zp/summary.txt
done
exit 0
