# round 3 (ll): the forces pass at 3 waves/SIMD without spills (LPE_FORCES_MINW=3 variant) vs the shipped 4 waves/SIMD
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03ll_snap.log 2>&1 || exit 1
for rep in 1 2 3; do
  for v in little-physics-engine_amd/liblpe_hip.so profiles/_var/liblpe_minw3.so; do
    LPE_LIB=$v TOPK=6 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03ll_rates.txt 2>&1 || exit 1
  done
done
