# round 6 (f): evidence on this round's library: PMC passes (traffic, VALU, density microbench) and the drop-in timed through the EnTT harness
mkdir -p gpurun_out/r06f
export TMPDIR=/tmp
bash profiles/pmc_collect.sh gpurun_out/r06f/pmc || exit 1
SQ2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $SQ2 --output-format csv -d gpurun_out/r06f/pmc -o M_sq2 -- python -u profiles/snapshot.py --load 20 > gpurun_out/r06f/pmc/M_sq2.log 2>&1; rc=$?; echo "M_sq2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python profiles/pmc_kernels.py gpurun_out/r06f/pmc/M_sq1_counter_collection.csv --last 50 --kernels k_density,k_forces_couple,k_pgs_stripes > gpurun_out/r06f/pmc/M_sq1_kernels.json || exit 1
python profiles/pmc_kernels.py gpurun_out/r06f/pmc/M_sq2_counter_collection.csv --last 50 --kernels k_density,k_forces_couple,k_pgs_stripes > gpurun_out/r06f/pmc/M_sq2_kernels.json || exit 1
timeout -k 10 900 python -u profiles/dropin_timing.py > gpurun_out/r06f/dropin.json 2> gpurun_out/r06f/dropin.err; rc=$?; echo "dropin rc=$rc"; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/r06f/pmc/*counter_collection.csv.big
exit 0
