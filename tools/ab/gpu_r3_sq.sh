# Round 3: where do C4's pull waves spend their cycles?  SQ counters of k_pull / k_pull_young
# (one PMC pass; the profiler serialises the two kernels).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 500 rocprofv3 --kernel-include-regex "k_pull" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d $R/gpurun_out/r3_sq_c4 -o run --output-format csv -- python $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r3_sq_c4.json 2> $R/gpurun_out/r3_sq_c4.err || { echo "sq failed"; tail -3 $R/gpurun_out/r3_sq_c4.err; exit 1; }
echo sq ok
timeout -s KILL 500 rocprofv3 --kernel-include-regex "k_pull" --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE -d $R/gpurun_out/r3_ta_c4 -o run --output-format csv -- python $R/bench.py --steps 4 --warmup 2 --no-cpu-baseline > $R/gpurun_out/r3_ta_c4.json 2> $R/gpurun_out/r3_ta_c4.err || { echo "ta failed"; tail -3 $R/gpurun_out/r3_ta_c4.err; exit 1; }
echo ta ok
