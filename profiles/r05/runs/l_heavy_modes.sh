# round 5 (l): heavy tiles on / off, multi-tick vs one-tick calls on the settled metric scene
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05l_snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
for rep in 1 2; do
  timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05l_modes.jsonl 2>> gpurun_out/r05l_err.log; rc=$?; ok $rc
  LPE_NO_HEAVY=1 timeout -k 10 200 python -u profiles/heavy_modes.py >> gpurun_out/r05l_modes.jsonl 2>> gpurun_out/r05l_err.log; rc=$?; ok $rc
done
exit 0
