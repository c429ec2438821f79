# round 6 (z8, after the coupling constants in LDS and the filed-block / permute round trips): the final library -- rocprofv3 over the bench command (its per-kernel window, stamped), the PMC passes, the drop-in timing
mkdir -p gpurun_out/r06g
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/r06g_prof -o bench -- python3 bench.py --no-extras --no-density-microbench --no-cpu-baseline --steps 50 > gpurun_out/r06g/bench_under_rocprof.json 2> gpurun_out/r06g/prof.log; rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
db=$(ls /tmp/r06g_prof/*.db | head -1)
python3 profiles/rocpd_summary.py $db --window-kernel k_forces_couple --window 500 --json gpurun_out/r06g/rocprof_window.json > gpurun_out/r06g/kernel_stats_bench_window.txt 2>&1 || exit 1
python3 profiles/rocpd_summary.py $db > gpurun_out/r06g/kernel_stats_bench_all.txt 2>&1 || exit 1
rm -rf /tmp/r06g_prof
bash profiles/pmc_collect.sh gpurun_out/r06g/pmc || exit 1
SQ2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $SQ2 --output-format csv -d gpurun_out/r06g/pmc -o M_sq2 -- python -u profiles/snapshot.py --load 20 > gpurun_out/r06g/pmc/M_sq2.log 2>&1; rc=$?; echo "M_sq2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python profiles/pmc_kernels.py gpurun_out/r06g/pmc/M_sq1_counter_collection.csv --last 50 --kernels k_density,k_forces_couple,k_pgs_stripes > gpurun_out/r06g/pmc/M_sq1_kernels.json || exit 1
python profiles/pmc_kernels.py gpurun_out/r06g/pmc/M_sq2_counter_collection.csv --last 50 --kernels k_density,k_forces_couple,k_pgs_stripes > gpurun_out/r06g/pmc/M_sq2_kernels.json || exit 1
timeout -k 10 900 python -u profiles/dropin_timing.py > gpurun_out/r06g/dropin.json 2> gpurun_out/r06g/dropin.err; rc=$?; echo "dropin rc=$rc"; [ $rc -eq 0 ] || exit $rc
exit 0
