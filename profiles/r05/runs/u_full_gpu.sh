# round 5 (u): the whole GPU suite and smoke on the tile-scheduling library
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r05u_gpu.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05u_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; exit $rc
