# round 4 (z): end-of-round evidence, part 4 (the final library): the drop-in timed through the EnTT host harness
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u profiles/dropin_timing.py > gpurun_out/r04z_dropin.json 2> gpurun_out/r04z_dropin.err || exit 1
