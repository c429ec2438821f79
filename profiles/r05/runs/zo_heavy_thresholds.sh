# round 5 (zo): the tile filing's class thresholds (quarters >= Q pairs, halves >= H): forces / density kernel times and tick rates at settled M
mkdir -p gpurun_out/r05zo
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zo/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
for qh in 512,256 768,384 1024,512 384,192 640,256 512,384; do
  q=${qh%,*}; h=${qh#*,}
  LPE_HEAVY_Q=$q LPE_HEAVY_H=$h timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05zo_$q_$h -o run -- python3 -u profiles/heavy_modes.py >> gpurun_out/r05zo/modes.jsonl 2> gpurun_out/r05zo/err_$q.log; rc=$?; echo "$q $h rc=$rc"; ok $rc
  f=$(find /tmp/r05zo_$q_$h -name '*kernel_stats.csv')
  python3 -c "
import csv,sys
rows={r['Name'].split('(')[0]:r for r in csv.DictReader(open('$f'))}
print('Q $q H $h', {k.split('::')[-1]: round(float(rows[k]['AverageNs'])/1e3,2) for k in rows if any(x in k for x in ('k_forces_couple','k_density<true>','k_scan_rows'))})" >> gpurun_out/r05zo/summary.txt
  rm -rf /tmp/r05zo_$q_$h
done
exit 0
