# round 5 (zr): striped-solver stamps on the live C1 stack (560 ticks in, as small_probe.py times it)
mkdir -p gpurun_out/r05zr
LIVE=C1 LPE_LIB=profiles/r05/var/liblpe_pt.so timeout -k 10 120 python -u profiles/stripe_trace.py > gpurun_out/r05zr/c1_live_stripe_trace.txt 2>&1; echo rc=$?
