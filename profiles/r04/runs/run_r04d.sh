# round 4 (d): where the 1-rank slab's wall goes: transport skipped (1 rank), forced RCCL call, loopback
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u profiles/slab_probe.py --loop --timing > gpurun_out/r04d_slab1.json 2> gpurun_out/r04d_slab1.err || exit 1
LPE_SLAB_FORCE_XCHG=1 timeout -k 10 300 python -u profiles/slab_probe.py > gpurun_out/r04d_slab1_force.json 2> gpurun_out/r04d_slab1_force.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04d_trace -o slab1 -- python3 -u profiles/slab_probe.py --prep 100 --ticks 20 --rounds 1 > gpurun_out/r04d_trace.log 2>&1 || exit 1
