# round 3 (f): forces-pass ablations (profiling variants, not bit-exact): phase traces and tick rates
mkdir -p gpurun_out
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03f_snap.log 2>&1 || exit 1
for v in ft ftfd ftnc ftnn; do
  echo "== $v" >> gpurun_out/r03f_ftrace.txt
  LPE_LIB=profiles/_var/liblpe_$v.so timeout -k 10 60 python -u profiles/forces_phase_trace.py >> gpurun_out/r03f_ftrace.txt 2>&1 || exit 1
done
for v in little-physics-engine_amd/liblpe_hip.so profiles/_var/liblpe_fd.so profiles/_var/liblpe_nc.so profiles/_var/liblpe_nn.so; do
  LPE_LIB=$v TOPK=12 timeout -k 10 60 python -u profiles/snapshot.py --load 400 >> gpurun_out/r03f_rates.txt 2>&1 || exit 1
done
