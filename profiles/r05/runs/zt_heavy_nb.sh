# round 5 (zt): tiles without coupling pairs but long neighbour lists filed as whole tiles (dispatched early): forces kernel time by threshold
mkdir -p gpurun_out/r05zt
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zt/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
for nb in 1073741824 3000 3500 4000 2600 1073741824; do
  LPE_HEAVY_NB=$nb timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05zt_$nb -o run -- python3 -u profiles/heavy_modes.py >> gpurun_out/r05zt/modes.jsonl 2> gpurun_out/r05zt/err_$nb.log; rc=$?; echo "$nb rc=$rc"; ok $rc
  f=$(find /tmp/r05zt_$nb -name '*kernel_stats.csv')
  python3 -c "
import csv,sys
rows={r['Name'].split('(')[0]:r for r in csv.DictReader(open('$f'))}
print('NB $nb', {k.split('::')[-1]: round(float(rows[k]['AverageNs'])/1e3,2) for k in rows if any(x in k for x in ('k_forces_couple','k_density<true>'))})" >> gpurun_out/r05zt/summary.txt
  rm -rf /tmp/r05zt_$nb
done
exit 0
