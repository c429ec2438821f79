# round 3 (o): stripe workgroup size A/B (rigid microbench, C1/C3/M rates)
mkdir -p gpurun_out
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03o_snap.log 2>&1 || exit 1
for v in little-physics-engine_amd/liblpe_hip.so profiles/_var/liblpe_st128.so profiles/_var/liblpe_st64.so; do
  LPE_LIB=$v timeout -k 10 120 python -u profiles/rigid_ab.py >> gpurun_out/r03o_ab.txt 2>&1 || exit 1
  LPE_LIB=$v timeout -k 10 180 python -u profiles/config_ab.py --m >> gpurun_out/r03o_ab.txt 2>&1 || exit 1
done
