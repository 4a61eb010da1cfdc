# Round 4: where k_pull_young's cycles go on the final kernels: the phase-stamp build (cycles per
# phase of the node loop) and one SQ pass (VALU / LDS / SALU issue and activity) on a C4 shard.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_ys/libgossip.so GOSSIP_YOUNG_OVERLAP=0 timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4p_ys.json 2> gpurun_out/r4p_ys.err || { tail -5 gpurun_out/r4p_ys.err; exit 1; }
python tools/ab_line.py ys_seq gpurun_out/r4p_ys.json
grep young_stamps gpurun_out/r4p_ys.err | tail -2
cd /tmp && export TMPDIR=/tmp
B2="python $R/bench.py --rehearse-shards 2 --steps 5 --warmup 5 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull_young" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS -d $R/gpurun_out/r4p_sq -o run --output-format csv -- $B2 > $R/gpurun_out/r4p_sq.json 2> $R/gpurun_out/r4p_sq.err || { echo "sq failed"; tail -3 $R/gpurun_out/r4p_sq.err; exit 1; }
python $R/tools/pmc_counters.py --timed 5 --kernel "k_pull_young" $R/gpurun_out/r4p_sq/run_counter_collection.csv
