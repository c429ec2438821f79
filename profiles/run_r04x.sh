# round 4 (x): where the pile blocks' coupling phase goes: forces trace of the shipped arithmetic, without the rigid accumulators' atomics (LPE_XP_NOXACC), without the impulse term (LPE_XP_NOIMP) -- timing-only variants
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r04x_snap.log 2>&1 || exit 1
for v in ft ftnx ftni; do
  LPE_LIB=profiles/_var/liblpe_$v.so timeout -k 10 120 python -u profiles/forces_trace.py > gpurun_out/r04x_ftrace_$v.txt 2>&1 || exit 1
done
