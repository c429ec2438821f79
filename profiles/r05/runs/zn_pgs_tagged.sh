# round 5 (zn): the PGS stripes' tagged hand-over (values carry their epoch) vs flags + reload: parity, rigid microbench, kernel times, tick rates
mkdir -p gpurun_out/r05zn
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 900 python -u -m pytest tests/test_rigid_gpu.py tests/test_configs_gpu.py tests/test_world_gpu.py tests/test_jacobi_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05zn/parity.log 2>&1; rc=$?; echo "parity rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
for v in new prev new prev; do
  if [ $v = prev ]; then export LPE_LIB=profiles/r05/var/liblpe_prev.so; else unset LPE_LIB; fi
  timeout -k 10 200 python -u profiles/rigid_ab.py >> gpurun_out/r05zn/rigid_ab.jsonl 2>> gpurun_out/r05zn/err.log; rc=$?; ok $rc
done
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zn/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
for v in new nofuse prev; do
  unset LPE_LIB LPE_NO_RBIN_FUSION
  if [ $v = prev ]; then export LPE_LIB=profiles/r05/var/liblpe_prev.so; fi
  if [ $v = nofuse ]; then export LPE_NO_RBIN_FUSION=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05zn_$v -o run -- python3 -u profiles/heavy_modes.py >> gpurun_out/r05zn/modes_$v.jsonl 2> gpurun_out/r05zn/$v.log; rc=$?; echo "$v rc=$rc"; ok $rc
  cp $(find /tmp/r05zn_$v -name '*kernel_stats.csv') gpurun_out/r05zn/${v}_kernel_stats.csv; rm -rf /tmp/r05zn_$v
  python3 -c "
import csv,sys
rows={r['Name'].split('(')[0]:r for r in csv.DictReader(open('gpurun_out/r05zn/${v}_kernel_stats.csv'))}
print('$v', {k.split('::')[-1]: round(float(rows[k]['AverageNs'])/1e3,2) for k in rows if any(x in k for x in ('k_pgs_stripes','k_pos_stripes','k_forces_couple','k_rbin','k_scan_reduce','k_scan_final'))})" >> gpurun_out/r05zn/summary.txt
done
unset LPE_LIB LPE_NO_RBIN_FUSION
for v in new prev new prev; do
  if [ $v = prev ]; then export LPE_LIB=profiles/r05/var/liblpe_prev.so; else unset LPE_LIB; fi
  timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05zn/rates_$v.jsonl 2>> gpurun_out/r05zn/err.log; rc=$?; ok $rc
done
exit 0
