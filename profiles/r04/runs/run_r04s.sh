# round 4 (s): k_group_colour stage trace (list compaction / barrier / chain) on the pile fixture, C1, C3
mkdir -p gpurun_out
export TMPDIR=/tmp
LPE_LIB=profiles/_var/liblpe_pt.so timeout -k 10 200 python -u profiles/colour_trace.py > gpurun_out/r04s_ctrace.txt 2>&1 || exit 1
