# round 5 (zj): the rigid bins in one launch (k_rbin_build, histogram of up to 38,912 bins in LDS) vs four launches: parity, kernel times, tick rates
mkdir -p gpurun_out/r05zj
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py tests/test_world_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05zj/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zj/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
for v in new nofuse; do
  unset LPE_NO_RBIN_FUSION
  if [ $v = nofuse ]; then export LPE_NO_RBIN_FUSION=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05zj_$v -o run -- python3 -u profiles/heavy_modes.py >> gpurun_out/r05zj/modes_$v.jsonl 2> gpurun_out/r05zj/$v.log; rc=$?; echo "$v rc=$rc"; ok $rc
  cp $(find /tmp/r05zj_$v -name '*kernel_stats.csv') gpurun_out/r05zj/${v}_kernel_stats.csv; rm -rf /tmp/r05zj_$v
  python3 -c "
import csv,sys
rows={r['Name'].split('(')[0]:r for r in csv.DictReader(open('gpurun_out/r05zj/${v}_kernel_stats.csv'))}
print('$v', {k.split('::')[-1]: (rows[k]['Calls'], round(float(rows[k]['AverageNs'])/1e3,2)) for k in rows if any(x in k for x in ('k_rbin','k_scan_reduce','k_scan_final','k_pgs_stripes','k_pos_stripes'))})" >> gpurun_out/r05zj/summary.txt
done
unset LPE_NO_RBIN_FUSION
for v in new nofuse new nofuse; do
  unset LPE_NO_RBIN_FUSION
  if [ $v = nofuse ]; then export LPE_NO_RBIN_FUSION=1; fi
  timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05zj/rates_$v.jsonl 2>> gpurun_out/r05zj/err.log; rc=$?; ok $rc
done
exit 0
