# round 5 (c): PGS / position solver -- single-wave schedule for steps of up to 128 pairs (new) and the
# scalar row math (pgss, -DPGS_SCALAR=1) against the round-start library (base): rigid tests, rigid
# microbench on the pile fixture, C1/C3/C2 and settled-M tick rates, alternating
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 400 python -u -m pytest tests/test_rigid_gpu.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r05c_rigid.log 2>&1; rc=$?; echo "rigid rc=$rc"; ok $rc
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05c_snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
for rep in 1 2; do
  for v in base new pgss; do
    if [ $v = new ]; then L=""; else L=profiles/r05/var/liblpe_$v.so; fi
    LPE_LIB=$L timeout -k 10 120 python -u profiles/rigid_ab.py >> gpurun_out/r05c_rigid_ab.jsonl 2>> gpurun_out/r05c_err.log; rc=$?; ok $rc
    LPE_LIB=$L timeout -k 10 200 python -u profiles/config_ab.py --m >> gpurun_out/r05c_config_ab.jsonl 2>> gpurun_out/r05c_err.log; rc=$?; ok $rc
  done
done
exit 0
