# round 3 (ee): the tick density pass in plain block order (LPE_DENSITY_PLAIN variant) vs XCD-contiguous: settled rates
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03ee_snap.log 2>&1 || exit 1
for rep in 1 2; do
  for v in little-physics-engine_amd/liblpe_hip.so profiles/_var/liblpe_dplain.so; do
    LPE_LIB=$v TOPK=8 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03ee_rates.txt 2>&1 || exit 1
  done
done
