# round 5 (zw): the density and forces passes at wave priority 2 vs the previous library: in-tick kernel times and tick rates
mkdir -p gpurun_out/r05zw
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zw/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
for v in new prev; do
  unset LPE_LIB
  if [ $v = prev ]; then export LPE_LIB=profiles/r05/var/liblpe_prev.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05zw_$v -o run -- python3 -u profiles/heavy_modes.py >> gpurun_out/r05zw/modes_$v.jsonl 2> gpurun_out/r05zw/$v.log; rc=$?; echo "$v rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
  cp $(find /tmp/r05zw_$v -name '*kernel_stats.csv') gpurun_out/r05zw/${v}_kernel_stats.csv; rm -rf /tmp/r05zw_$v
  python3 -c "
import csv
rows={r['Name'].split('(')[0]:r for r in csv.DictReader(open('gpurun_out/r05zw/${v}_kernel_stats.csv'))}
print('$v', {k.split('::')[-1]: round(float(rows[k]['AverageNs'])/1e3,2) for k in rows if any(x in k for x in ('k_pgs_stripes','k_pos_stripes','k_density','k_forces_couple','k_scan_rows','k_bucket_permute'))})" >> gpurun_out/r05zw/summary.txt
done
unset LPE_LIB
for v in new prev new prev; do
  unset LPE_LIB
  if [ $v = prev ]; then export LPE_LIB=profiles/r05/var/liblpe_prev.so; fi
  timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05zw/rates_$v.jsonl 2>> gpurun_out/r05zw/err.log; rc=$?; ok $rc; [ $rc -eq 0 ] || exit 1
done
exit 0
