# round 4 (j): parity of the wave-uniform group colouring; forces image trace; stripe solver trace; rigid microbench
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rigid_gpu.py tests/test_world_gpu.py -q -x --timeout 180 --timeout-method thread > gpurun_out/r04j_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"
if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r04j_snap.log 2>&1 || exit 1
LPE_LIB=profiles/_var/liblpe_ft.so timeout -k 10 120 python -u profiles/forces_trace.py > gpurun_out/r04j_ftrace.txt 2>&1 || exit 1
LPE_LIB=profiles/_var/liblpe_pt.so timeout -k 10 120 python -u profiles/stripe_trace.py > gpurun_out/r04j_strace.txt 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --no-cpu-baseline > gpurun_out/r04j_bench.json 2> gpurun_out/r04j_bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d /tmp/r04j_prof_slab1 -o slab1 -- python3 profiles/slab_probe.py --only slab1 --prep 300 --ticks 30 --rounds 1 > gpurun_out/r04j_prof_slab1.log 2>&1 || exit 1
db=$(ls /tmp/r04j_prof_slab1/*.db | head -1)
python3 profiles/rocpd_summary.py $db --api 25 --timeline 400 --skip 30000 > gpurun_out/r04j_prof_slab1.txt 2>&1 || exit 1
