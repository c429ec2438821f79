# round 3 (v): the full -m gpu suite on the bucket build; PGS step-cost variants (empty steps / no row math) on the pile fixture
mkdir -p gpurun_out
ok() { local rc=$1; if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then echo "stop: rc=$rc"; exit $rc; fi; return 0; }
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03v_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; ok $rc; [ $rc -eq 0 ] || exit 1
for v in little-physics-engine_amd/liblpe_hip.so profiles/_var/liblpe_pgsempty.so profiles/_var/liblpe_pgsnomath.so; do
  LPE_LIB=$v timeout -k 10 120 python -u profiles/rigid_ab.py >> gpurun_out/r03v_ab.txt 2>&1 || exit 1
done
