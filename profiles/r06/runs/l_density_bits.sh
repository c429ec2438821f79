#!/bin/bash
# Density: neighbours filed from per-window bits (default) against one ring
# store per candidate (LPE_DENSITY_RING=1), alternating, from the settled
# snapshot; then the density / config parity tests.
set -e
mkdir -p gpurun_out/db
timeout -k 10 120 python3 profiles/snapshot.py --save 3000 > gpurun_out/db/snap.log 2>&1
for rep in 1 2; do
  TOPK=12 timeout -k 10 60 python3 profiles/snapshot.py --load 1200 | sed 's/^/bits /' >> gpurun_out/db/ab.txt 2>&1
  LPE_DENSITY_RING=1 TOPK=12 timeout -k 10 60 python3 profiles/snapshot.py --load 1200 | sed 's/^/ring /' >> gpurun_out/db/ab.txt 2>&1
done
cat gpurun_out/db/ab.txt


