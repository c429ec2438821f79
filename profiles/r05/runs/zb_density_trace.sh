# round 5 (zb): per-tile phase trace of the tick's density pass (settled M)
mkdir -p gpurun_out/r05zb
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zb/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
LPE_LIB=profiles/r05/var/liblpe_ft.so timeout -k 10 120 python -u profiles/density_trace.py > gpurun_out/r05zb/density_trace.txt 2>&1; rc=$?; echo "trace rc=$rc"; ok $rc
LPE_NO_HEAVY=1 LPE_LIB=profiles/r05/var/liblpe_ft.so timeout -k 10 120 python -u profiles/density_trace.py > gpurun_out/r05zb/density_trace_noheavy.txt 2>&1; rc=$?; echo "trace rc=$rc"; ok $rc
exit 0
