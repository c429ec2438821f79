# round 3 PMC passes (one counter group per rocprofv3 run, MI355X_MICROARCH.md):
# the settled metric scene (snapshot, last ticks) and the 16.7M density microbench
mkdir -p gpurun_out/r03_pmc
export TMPDIR=/tmp
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > gpurun_out/r03_pmc/snap.log 2>&1 || exit 1
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
SQ2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
run() {  # name, counters, command...
  local n=$1 c=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r03_pmc -o $n -- "$@" > gpurun_out/r03_pmc/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run M_sq1 "$SQ1" python -u profiles/snapshot.py --load 20
run M_sq2 "$SQ2" python -u profiles/snapshot.py --load 20
run M_fetch "FETCH_SIZE" python -u profiles/snapshot.py --load 20
run M_write "WRITE_SIZE" python -u profiles/snapshot.py --load 20
run D_sq1 "$SQ1" python -u profiles/density_micro.py --reps 3
run D_sq2 "$SQ2" python -u profiles/density_micro.py --reps 3
run D_fetch "FETCH_SIZE" python -u profiles/density_micro.py --reps 3
run D_write "WRITE_SIZE" python -u profiles/density_micro.py --reps 3
