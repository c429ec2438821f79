# round 3 (u): helper-term caps raised (256 particles / 1024 items per block): A/B on the settled scene + phase traces
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/m240.py > gpurun_out/r03u_m240.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_sph_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03u_pytest.log 2>&1 || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03u_snap.log 2>&1 || exit 1
for rep in 1 2; do
  for t in 0 16 24; do
    echo "T=$t" >> gpurun_out/r03u_rates.txt
    LPE_FORCES_T=$t TOPK=6 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03u_rates.txt 2>&1 || exit 1
  done
done
for t in 0 24; do
  echo "T=$t" >> gpurun_out/r03u_ftrace.txt
  LPE_FORCES_T=$t LPE_LIB=profiles/_var/liblpe_ft.so timeout -k 10 60 python -u profiles/forces_phase_trace.py >> gpurun_out/r03u_ftrace.txt 2>&1 || exit 1
done
