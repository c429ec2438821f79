#!/bin/bash
# k_forces_couple's SGPR spills: the coupling constants (cpl) and the next
# kick's parameters (cplkn) read from LDS copies instead of kernel-argument
# SGPRs, against the previous library, alternating from the settled snapshot.
set -e
mkdir -p gpurun_out/xs
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/xs/snap.log 2>&1
for rep in 1 2 3; do
  for v in prev cpl cplkn; do
    LPE_LIB=profiles/_var/liblpe_$v.so TOPK=6 timeout -k 10 60 python3 profiles/snapshot.py --load 2400 | sed "s/^/$v /" >> gpurun_out/xs/ab.txt 2>&1
  done
done
cat gpurun_out/xs/ab.txt
