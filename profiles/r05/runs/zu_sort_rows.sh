# round 5 (zu): the row scan and the bucket permute as one launch (k_sort_rows) vs the two (LPE_NO_SORT_ROWS=1): parity, kernel times, tick rates
mkdir -p gpurun_out/r05zu
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 700 python -u -m pytest tests/test_sph_gpu.py tests/test_configs_gpu.py tests/test_world_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05zu/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zu/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
for v in new old; do
  unset LPE_NO_SORT_ROWS
  if [ $v = old ]; then export LPE_NO_SORT_ROWS=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05zu_$v -o run -- python3 -u profiles/heavy_modes.py >> gpurun_out/r05zu/modes_$v.jsonl 2> gpurun_out/r05zu/$v.log; rc=$?; echo "$v rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
  cp $(find /tmp/r05zu_$v -name '*kernel_stats.csv') gpurun_out/r05zu/${v}_kernel_stats.csv; rm -rf /tmp/r05zu_$v
  python3 -c "
import csv
rows={r['Name'].split('(')[0]:r for r in csv.DictReader(open('gpurun_out/r05zu/${v}_kernel_stats.csv'))}
print('$v', {k.split('::')[-1]: round(float(rows[k]['AverageNs'])/1e3,2) for k in rows if any(x in k for x in ('k_sort_rows','k_scan_rows','k_bucket_permute','k_density','k_forces_couple'))})" >> gpurun_out/r05zu/summary.txt
done
for v in new old new old; do
  unset LPE_NO_SORT_ROWS
  if [ $v = old ]; then export LPE_NO_SORT_ROWS=1; fi
  timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05zu/rates_$v.jsonl 2>> gpurun_out/r05zu/err.log; rc=$?; ok $rc; [ $rc -eq 0 ] || exit 1
done
exit 0
