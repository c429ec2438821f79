# round 5 (e): forces per-block traces (one launch, clean slots) with and without heavy tiles, with and
# without the rigid accumulators' atomics (timing only); tick rates base / new / new without heavy tiles
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05e_snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
for v in ft ftna; do
  LPE_LIB=profiles/r05/var/liblpe_$v.so timeout -k 10 120 python -u profiles/forces_trace.py > gpurun_out/r05e_trace_${v}_heavy.txt 2>&1; rc=$?; ok $rc
  LPE_NO_HEAVY=1 LPE_LIB=profiles/r05/var/liblpe_$v.so timeout -k 10 120 python -u profiles/forces_trace.py > gpurun_out/r05e_trace_${v}_plain.txt 2>&1; rc=$?; ok $rc
done
for rep in 1 2; do
  LPE_LIB=profiles/r05/var/liblpe_base.so timeout -k 10 200 python -u profiles/config_ab.py --m >> gpurun_out/r05e_config_ab.jsonl 2>> gpurun_out/r05e_err.log; rc=$?; ok $rc
  timeout -k 10 200 python -u profiles/config_ab.py --m >> gpurun_out/r05e_config_ab.jsonl 2>> gpurun_out/r05e_err.log; rc=$?; ok $rc
  LPE_NO_HEAVY=1 timeout -k 10 200 python -u profiles/config_ab.py --m | sed 's/"lib": ""/"lib": "new, LPE_NO_HEAVY=1"/' >> gpurun_out/r05e_config_ab.jsonl 2>> gpurun_out/r05e_err.log; rc=$?; ok $rc
done
exit 0
