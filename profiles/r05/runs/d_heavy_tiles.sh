# round 5 (d): forces pass with heavy tiles run as quarter blocks -- SPH / world / config / slab parity,
# the per-block trace at settled M, tick rates against the round-start library (base), alternating
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 900 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py tests/test_configs_gpu.py tests/test_slab_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r05d_parity.log 2>&1; rc=$?; echo "parity rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05d_snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
LPE_LIB=profiles/r05/var/liblpe_ft.so timeout -k 10 120 python -u profiles/forces_trace.py > gpurun_out/r05d_forces_trace.txt 2>&1; rc=$?; echo "ftrace rc=$rc"; ok $rc
for rep in 1 2; do
  for v in base new; do
    if [ $v = new ]; then L=""; else L=profiles/r05/var/liblpe_$v.so; fi
    LPE_LIB=$L timeout -k 10 200 python -u profiles/config_ab.py --m >> gpurun_out/r05d_config_ab.jsonl 2>> gpurun_out/r05d_err.log; rc=$?; ok $rc
  done
done
exit 0
