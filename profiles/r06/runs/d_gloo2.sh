# round 6 (d): the N-GPU bench line rehearsed with 2 gloo ranks on one GPU, capped cells (the new default)
mkdir -p gpurun_out/r06d
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --gpus 2 --transport gloo --steps 10 --warmup 3 --prep 60 --strong-prep 20 --no-cpu-baseline > gpurun_out/r06d/bench_gloo2.json 2> gpurun_out/r06d/bench_gloo2.err; rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/r06d/bench_gloo2.err
exit $rc
