# round 3 (k): the whole -m gpu suite on the current tree
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r03k_pytest.log 2>&1; echo "pytest rc=$?"
