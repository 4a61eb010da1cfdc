# PMC exploration of the C3 bench's k_pull (one counter group per run, counters only)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -d $R/gpurun_out/pmc2_$i -o run --output-format csv -- python $R/bench.py --no-cpu-baseline --steps 20 --warmup 30 > /dev/null 2>$R/gpurun_out/pmc2_$i.err || { echo "pass $i ($grp) failed"; tail -3 $R/gpurun_out/pmc2_$i.err; exit 1; }
done
cd $R
python tools/pmc_counters.py --timed 20 gpurun_out/pmc2_*/run_counter_collection.csv | tee gpurun_out/pmc2.json
