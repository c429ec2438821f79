# round 3 (kk): density walks read 12 of a record's 16 LDS bytes (ds_read_b96): parity, settled rates and the
# density microbench (variant profiles/_var/liblpe_b96.so) against the shipped build
mkdir -p gpurun_out
export TMPDIR=/tmp
LPE_LIB=profiles/_var/liblpe_b96.so timeout -k 10 400 python -u -m pytest tests/test_sph_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03kk_pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03kk_snap.log 2>&1 || exit 1
for rep in 1 2; do
  for v in little-physics-engine_amd/liblpe_hip.so profiles/_var/liblpe_b96.so; do
    LPE_LIB=$v TOPK=6 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03kk_rates.txt 2>&1 || exit 1
    LPE_LIB=$v timeout -k 10 120 python -u profiles/density_micro.py --reps 5 >> gpurun_out/r03kk_dm.txt 2>&1 || exit 1
  done
done
