# PMC passes of the shipped build (one counter group per rocprofv3 run, MI355X_MICROARCH.md):
# the settled metric scene (snapshot, last ticks) and the 16.7M density microbench.
#   bash profiles/pmc_collect.sh OUTDIR      (on the GPU box; OUTDIR under gpurun_out/)
# writes OUTDIR/{pmc_traffic,pmc_valu,pmc_density_pair}.json stamped with the library's sha256
set -u
OUT=${1:-gpurun_out/pmc_final}
mkdir -p $OUT
export TMPDIR=/tmp
LIB=little-physics-engine_amd/liblpe_hip.so
timeout -k 10 120 python -u profiles/snapshot.py --save 3000 > $OUT/snap.log 2>&1 || exit 1
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
SQ2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
run() {  # name, counters, command...
  local n=$1 c=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d $OUT -o $n -- "$@" > $OUT/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
run M_sq1 "$SQ1" python -u profiles/snapshot.py --load 20
run M_fetch "FETCH_SIZE" python -u profiles/snapshot.py --load 20
run M_write "WRITE_SIZE" python -u profiles/snapshot.py --load 20
run D_sq1 "$SQ1" python -u profiles/density_micro.py --reps 3
run D_sq2 "$SQ2" python -u profiles/density_micro.py --reps 3
run D_fetch "FETCH_SIZE" python -u profiles/density_micro.py --reps 3
run D_write "WRITE_SIZE" python -u profiles/density_micro.py --reps 3
timeout -k 10 120 python -u profiles/density_micro.py --reps 5 > $OUT/density_micro.json 2>&1 || exit 1
python profiles/pmc_traffic.py $OUT/M_fetch_counter_collection.csv $OUT/M_write_counter_collection.csv $OUT/pmc_traffic.json --last 50 --lib $LIB > /dev/null || exit 1
python profiles/pmc_valu.py $OUT/M_sq1_counter_collection.csv $OUT/pmc_valu.json --last 50 --lib $LIB > /dev/null || exit 1
python - $OUT <<'PY'
import json, subprocess, sys
out = sys.argv[1]
d = json.loads(open(f"{out}/density_micro.json").read().strip().splitlines()[-1])
subprocess.check_call([sys.executable, "profiles/pmc_density.py", out, f"{out}/pmc_density_pair.json",
                       str(d["kernels_us"]["k_density"]), str(d["kernels_us"]["k_density_plan"]), "--lib",
                       "little-physics-engine_amd/liblpe_hip.so"])
PY
