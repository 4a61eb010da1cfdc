# Round 6: SQ counters of the C4 pull kernels at the driver's arguments, one
# PMC pass (rocprofv3 serialises the dispatches, so each kernel is measured alone), + the
# GPU clock (GRBM_GUI_ACTIVE); tools/pmc_counters.py averages the timed dispatches per kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
timeout -s KILL 420 rocprofv3 --kernel-include-regex "k_pull" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/r6i_sq -o run --output-format csv -- $B > $R/gpurun_out/r6i_sq.json 2> $R/gpurun_out/r6i_sq.err || { echo "sq pass failed"; tail -5 $R/gpurun_out/r6i_sq.err; exit 1; }
cd $R
F=$(ls gpurun_out/r6i_sq/*counter_collection.csv | head -1)
python tools/pmc_counters.py --timed 40 --kernel "k_pull<" $F > gpurun_out/r6i_sq_pull.json && cat gpurun_out/r6i_sq_pull.json
python tools/pmc_counters.py --timed 28 --kernel "k_pull_young" $F > gpurun_out/r6i_sq_young.json && cat gpurun_out/r6i_sq_young.json
