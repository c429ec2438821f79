# round 5 (zx): how much the prelaunched sub-step slows the PGS beside it: kernel times and tick rates with and without the prelaunch (LPE_NO_PRELAUNCH=1), same library
mkdir -p gpurun_out/r05zx
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zx/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
for v in pre nopre; do
  unset LPE_NO_PRELAUNCH
  if [ $v = nopre ]; then export LPE_NO_PRELAUNCH=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05zx_$v -o run -- python3 -u profiles/heavy_modes.py >> gpurun_out/r05zx/modes_$v.jsonl 2> gpurun_out/r05zx/$v.log; rc=$?; echo "$v rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
  cp $(find /tmp/r05zx_$v -name '*kernel_stats.csv') gpurun_out/r05zx/${v}_kernel_stats.csv; rm -rf /tmp/r05zx_$v
  python3 -c "
import csv
rows={r['Name'].split('(')[0]:r for r in csv.DictReader(open('gpurun_out/r05zx/${v}_kernel_stats.csv'))}
print('$v', {k.split('::')[-1]: round(float(rows[k]['AverageNs'])/1e3,2) for k in rows if any(x in k for x in ('k_pgs_stripes','k_pos_stripes','k_density','k_forces_couple','k_scan_rows','k_bucket_permute','k_kick_drift'))})" >> gpurun_out/r05zx/summary.txt
done
for v in pre nopre pre nopre; do
  unset LPE_NO_PRELAUNCH
  if [ $v = nopre ]; then export LPE_NO_PRELAUNCH=1; fi
  timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05zx/rates_$v.jsonl 2>> gpurun_out/r05zx/err.log; rc=$?; ok $rc; [ $rc -eq 0 ] || exit 1
done
exit 0
