# round 5 (zs): per-tile density and forces phase traces at C2 (64k-particle dam break, 30 ticks in), prelaunch off
mkdir -p gpurun_out/r05zs
SCENE=C2 LPE_NO_PRELAUNCH=1 LPE_LIB=profiles/r05/var/liblpe_ft.so timeout -k 10 120 python -u profiles/density_trace.py > gpurun_out/r05zs/c2_density_trace.txt 2>&1; echo rc=$?
