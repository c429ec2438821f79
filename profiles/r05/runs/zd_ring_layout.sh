# round 5 (zd): density neighbour-list ring entry-major (conflict-free 16-bit stores) vs lane-major: parity, kernel times (settled M)
mkdir -p gpurun_out/r05zd
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py tests/test_sph_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05zd/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zd/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
for v in new lane new lane; do
  if [ $v = lane ]; then export LPE_LIB=profiles/r05/var/liblpe_ringlane.so; else unset LPE_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05zd_$v -o run -- python3 -u profiles/heavy_modes.py >> gpurun_out/r05zd/modes_$v.jsonl 2> gpurun_out/r05zd/$v.log; rc=$?; echo "$v rc=$rc"; ok $rc
  cp $(find /tmp/r05zd_$v -name '*kernel_stats.csv') gpurun_out/r05zd/${v}_kernel_stats.csv; rm -rf /tmp/r05zd_$v
  python3 -c "
import csv,sys
rows={r['Name'].split('(')[0]:r for r in csv.DictReader(open('gpurun_out/r05zd/${v}_kernel_stats.csv'))}
print('$v', {k: round(float(rows[k]['AverageNs'])/1e3,2) for k in rows if any(x in k for x in ('k_density<true>','k_forces_couple'))})" >> gpurun_out/r05zd/summary.txt
done
exit 0
