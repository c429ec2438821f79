# round 4 (aa): the settled scene-M tick as a timeline (rocprofv3 kernel trace of the final library, two ticks of dispatches) -- idle gaps on the serial path
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r04aa_snap.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace -d /tmp/r04aa_tl -o tl -- python3 -u profiles/snapshot.py --load 30 > gpurun_out/r04aa_prof.log 2>&1 || exit 1
db=$(ls /tmp/r04aa_tl/*.db | head -1)
python3 profiles/rocpd_summary.py $db --timeline 170 --skip 1500 > gpurun_out/r04aa_timeline.txt 2>&1 || exit 1
