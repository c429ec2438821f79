#!/bin/bash
# Tile-scheduling class capacities (HALF_MAX full at scene M: T >= 256 tiles ran whole).
# Variants built by profiles/trace_build.sh sph NAME -DLPE_HALF_MAX=...; alternating A/B
# from the settled snapshot (snapshot.py --load: ticks/s + per-kernel HIP-event times).
set -e
mkdir -p gpurun_out/heavy
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/heavy/snap.log 2>&1
for rep in 1 2; do
  for v in default hv1 hv2 hv3; do
    if [ $v = default ]; then lib=""; else lib=profiles/_var/liblpe_$v.so; fi
    LPE_LIB=$lib TOPK=4 timeout -k 10 60 python3 profiles/snapshot.py --load 1200 >> gpurun_out/heavy/ab.txt 2>&1
  done
  LPE_LIB=profiles/_var/liblpe_hv1.so LPE_HEAVY_H=128 TOPK=4 timeout -k 10 60 python3 profiles/snapshot.py --load 1200 | sed 's/^/H128 /' >> gpurun_out/heavy/ab.txt 2>&1
  LPE_LIB=profiles/_var/liblpe_hv2.so LPE_HEAVY_Q=384 TOPK=4 timeout -k 10 60 python3 profiles/snapshot.py --load 1200 | sed 's/^/Q384 /' >> gpurun_out/heavy/ab.txt 2>&1
done
cat gpurun_out/heavy/ab.txt
LPE_LIB=profiles/_var/liblpe_dtl.so timeout -k 10 120 python3 profiles/density_sched.py gpurun_out/heavy/density_sched.npz > gpurun_out/heavy/density_sched.txt 2>&1
cat gpurun_out/heavy/density_sched.txt
