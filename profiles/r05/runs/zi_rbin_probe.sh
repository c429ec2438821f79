# round 5 (zi): the rigid-bin build's parameters in the settled-scene flow (LPE_DEBUG_RBIN)
mkdir -p gpurun_out/r05zi
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zi/snap.log 2>&1; echo snap rc=$?
LPE_DEBUG_RBIN=1 timeout -k 10 200 python -u profiles/heavy_modes.py > gpurun_out/r05zi/modes.log 2>&1; echo rc=$?
grep -m3 "rbin:" gpurun_out/r05zi/modes.log; grep -m3 "rbin:" gpurun_out/r05zi/snap.log
