# round 5 (zk): the settled scene-M tick as a timeline (rocprofv3 kernel trace of the current library) -- where the serial path goes
mkdir -p gpurun_out/r05zk
export TMPDIR=/tmp
timeout -k 10 200 python -u profiles/snapshot.py --save 3000 > gpurun_out/r05zk/snap.log 2>&1 || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace -d /tmp/r05zk_tl -o tl -- python3 -u profiles/snapshot.py --load 30 > gpurun_out/r05zk/prof.log 2>&1 || exit 1
db=$(ls /tmp/r05zk_tl/*.db | head -1)
python3 profiles/rocpd_summary.py $db --timeline 170 --skip 1500 > gpurun_out/r05zk/timeline.txt 2>&1 || exit 1
exit 0
