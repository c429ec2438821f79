# round 3 (n): kernel traces of the small configurations (C1, C2)
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03n_c1 -o trace -- python -u profiles/c1_run.py 200 C1 > gpurun_out/r03n_c1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r03n_c2 -o trace -- python -u profiles/c1_run.py 100 C2 > gpurun_out/r03n_c2.log 2>&1 || exit 1
