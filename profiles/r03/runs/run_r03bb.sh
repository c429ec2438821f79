# round 3 (bb): Barnes-Hut fold with the members' records loaded 8 ahead (parity + the bench's BH line);
# k_scan_rows stats reduced per wave before the LDS atomics (parity + settled rates)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_bh_gpu.py tests/test_sph_gpu.py tests/test_configs_gpu.py tests/test_host_mirror.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03bb_pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "
import json, sys, os
sys.path.insert(0, '.')
import bench
lpe = bench._load('lpe', os.path.join(bench.PKG, 'lpe.py')); scenes = bench._load('scenes', os.path.join(bench.PKG, 'scenes.py'))
print(json.dumps(bench.bh_bench(lpe, scenes, 0)))
" > gpurun_out/r03bb_bh.json 2>&1 || exit 1
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03bb_snap.log 2>&1 || exit 1
for rep in 1 2; do
  TOPK=12 timeout -k 10 60 python -u profiles/snapshot.py --load 600 >> gpurun_out/r03bb_rates.txt 2>&1 || exit 1
done
