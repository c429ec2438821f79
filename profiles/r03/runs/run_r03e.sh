# round 3 (e): forces-pass block order sweep (LPE_FORCES_CHUNK) on the settled metric scene
mkdir -p gpurun_out
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03e_snap.log 2>&1 || exit 1
for rep in 1 2; do
for c in 0 2 4 8 16 32; do
  echo "chunk=$c" >> gpurun_out/r03e_sweep.txt
  LPE_FORCES_CHUNK=$c TOPK=4 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03e_sweep.txt 2>&1 || exit 1
done
done
LPE_FORCES_CHUNK=8 timeout -k 10 300 python -u -m pytest tests/test_sph_gpu.py tests/test_world_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e_pytest.log 2>&1; echo "pytest rc=$?"
