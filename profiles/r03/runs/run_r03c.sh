# round 3 (c): kernel trace + stats of the settled metric scene (snapshot), for the tick timeline
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03c_snap.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03c_trace -o trace -- python -u profiles/snapshot.py --load 60 > gpurun_out/r03c_prof.log 2>&1 || exit 1
