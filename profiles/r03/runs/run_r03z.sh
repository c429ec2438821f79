# round 3 (z): rocprofv3 kernel stats of the settled metric scene (snapshot of 3000 ticks, 60 + 10 timed ticks) in the
# same process that prints the library's own HIP-event means: the two timing methods side by side
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03z_snap.log 2>&1 || exit 1
TOPK=40 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03z_stats -o snap -- python -u profiles/snapshot.py --load 60 > gpurun_out/r03z_prof.log 2>&1 || exit 1
TOPK=40 timeout -k 10 60 python -u profiles/snapshot.py --load 600 > gpurun_out/r03z_events.txt 2>&1 || exit 1
find gpurun_out/r03z_stats -name "*kernel_trace.csv" -size +20M -delete
