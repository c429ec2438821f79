# round 5 (zq): per-phase stamps of the striped solvers on the C1 stack fixture (one stripe) and on the metric pile
mkdir -p gpurun_out/r05zq
FIXTURE=rigid_C1_t120.npz LPE_LIB=profiles/r05/var/liblpe_pt.so timeout -k 10 120 python -u profiles/stripe_trace.py > gpurun_out/r05zq/c1_stripe_trace.txt 2>&1; echo rc=$?
LPE_LIB=profiles/r05/var/liblpe_pt.so timeout -k 10 120 python -u profiles/stripe_trace.py > gpurun_out/r05zq/pile_stripe_trace.txt 2>&1; echo rc=$?
timeout -k 10 200 python -u profiles/small_probe.py --scene C1 > gpurun_out/r05zq/small_c1.json 2>&1; echo rc=$?
