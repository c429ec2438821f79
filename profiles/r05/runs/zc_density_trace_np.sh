# round 5 (zc): density per-tile trace with the prelaunch off (the stamps are then the tick's last sub-step's, not the next tick's prelaunched, CU-masked pass)
mkdir -p gpurun_out/r05zc
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zc/snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
LPE_NO_PRELAUNCH=1 LPE_LIB=profiles/r05/var/liblpe_ft.so timeout -k 10 120 python -u profiles/density_trace.py > gpurun_out/r05zc/density_trace.txt 2>&1; rc=$?; echo "trace rc=$rc"; ok $rc
LPE_NO_PRELAUNCH=1 LPE_NO_HEAVY=1 LPE_LIB=profiles/r05/var/liblpe_ft.so timeout -k 10 120 python -u profiles/density_trace.py > gpurun_out/r05zc/density_trace_noheavy.txt 2>&1; rc=$?; echo "trace rc=$rc"; ok $rc
exit 0
