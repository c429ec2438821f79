# round 5 (zf): PMC passes of the shipped build (profiles/pmc_collect.sh) plus the SQ wait/LDS group on the settled scene, per kernel
export TMPDIR=/tmp
OUT=gpurun_out/r05zf
bash profiles/pmc_collect.sh $OUT || exit 1
SQ2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $SQ2 --output-format csv -d $OUT -o M_sq2 -- python -u profiles/snapshot.py --load 20 > $OUT/M_sq2.log 2>&1; rc=$?; echo "M_sq2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python profiles/pmc_kernels.py $OUT/M_sq1_counter_collection.csv --last 50 --kernels k_density,k_forces_couple,k_pgs_stripes > $OUT/M_sq1_kernels.json || exit 1
python profiles/pmc_kernels.py $OUT/M_sq2_counter_collection.csv --last 50 --kernels k_density,k_forces_couple,k_pgs_stripes > $OUT/M_sq2_kernels.json || exit 1
rm -f $OUT/*_counter_collection.csv.gz
exit 0
