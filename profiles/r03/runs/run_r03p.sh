# round 3 (p): stripe solver per-step times (PTRACE build) on the pile fixture
mkdir -p gpurun_out
LPE_LIB=profiles/_var/liblpe_pt.so timeout -k 10 120 python -u profiles/stripe_trace.py > gpurun_out/r03p_strace.txt 2>&1
