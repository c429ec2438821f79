# round 4 (f): the drop-in timed through the EnTT harness at scene M
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u profiles/dropin_timing.py > gpurun_out/r04f_dropin.json 2> gpurun_out/r04f_dropin.err || exit 1
