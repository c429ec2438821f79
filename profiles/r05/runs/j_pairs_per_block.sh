# round 5 (j): coupling pairs per forces block and the pair phase, without (ft) and with (ftc) per-stage stamps
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05j_snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
for v in ft ftc; do
  LPE_LIB=profiles/r05/var/liblpe_$v.so timeout -k 10 120 python -u profiles/forces_trace.py > gpurun_out/r05j_trace_$v.txt 2>&1; rc=$?; ok $rc
done
exit 0
