# round 5 (b): rigid reference fixtures at bench scale; C4@3000 parity; forces per-block trace at settled M;
# the N-rank bench line rehearsed with 2 ranks on one GPU over the host-staged gloo transport
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
timeout -k 10 400 python -u -m pytest tests/test_rigid_gpu.py -m gpu -v --timeout 300 --timeout-method thread -s > gpurun_out/r05b_rigid.log 2>&1; rc=$?; echo "rigid rc=$rc"; ok $rc
timeout -k 10 500 python -u -m pytest tests/test_configs_gpu.py -m gpu -v --timeout 400 --timeout-method thread -s -k "C4" > gpurun_out/r05b_c4.log 2>&1; rc=$?; echo "c4 rc=$rc"; ok $rc
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05b_snap.log 2>&1; rc=$?; echo "snap rc=$rc"; ok $rc
LPE_LIB=profiles/r05/var/liblpe_ft.so timeout -k 10 120 python -u profiles/forces_trace.py > gpurun_out/r05b_forces_trace.txt 2>&1; rc=$?; echo "ftrace rc=$rc"; ok $rc
timeout -k 10 400 python -u bench.py --gpus 2 --transport gloo --prep 300 --strong-prep 60 --warmup 3 --steps 10 > gpurun_out/r05b_bench2_gloo.json 2> gpurun_out/r05b_bench2_gloo.err; rc=$?; echo "bench2 rc=$rc"; ok $rc
exit 0
