# Round 3: why is the own-frontier dedup slower?  SQ/LDS counters of k_pull_young with
# young_own 0 / 1 (one C4 shard, 5 timed ticks), then A/B of young_skip and the k_pull builds with
# 4 / 12 loads in flight and a 5-wave register cap (shard 0 of 2).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for own in 0 1; do
  GOSSIP_YOUNG_OWN=$own timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $R/gpurun_out/r3w_sq$own -o run --output-format csv -- python $R/bench.py --rehearse-shards 2 --steps 5 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r3w_sq$own.json 2> $R/gpurun_out/r3w_sq$own.err || { echo "sq$own failed"; tail -3 $R/gpurun_out/r3w_sq$own.err; exit 1; }
  python $R/tools/pmc_counters.py --timed 5 --kernel k_pull_young $R/gpurun_out/r3w_sq$own/run_counter_collection.csv > $R/gpurun_out/r3w_sq${own}_young.txt
  python $R/tools/pmc_counters.py --timed 5 --kernel "k_pull<32" $R/gpurun_out/r3w_sq$own/run_counter_collection.csv > $R/gpurun_out/r3w_sq${own}_pull.txt
  echo "own=$own"; cat $R/gpurun_out/r3w_sq${own}_young.txt
done
cd $R
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3w_$name.json 2> gpurun_out/r3w_$name.err || { tail -5 gpurun_out/r3w_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3w_$name.json
}
L=$R/p2p-gossip-simulation-ns3_amd/lib
run skip0own0seq GOSSIP_YOUNG_OWN=0 GOSSIP_YOUNG_OVERLAP=0
run skip1own0seq GOSSIP_YOUNG_OWN=0 GOSSIP_YOUNG_SKIP=1 GOSSIP_YOUNG_OVERLAP=0
run skip1own1seq GOSSIP_YOUNG_OWN=1 GOSSIP_YOUNG_SKIP=1 GOSSIP_YOUNG_OVERLAP=0
run q4 GOSSIP_YOUNG_OWN=0 GOSSIP_LIB_PATH=$L/ab/q4.so
run q12 GOSSIP_YOUNG_OWN=0 GOSSIP_LIB_PATH=$L/ab/q12.so
run w5 GOSSIP_YOUNG_OWN=0 GOSSIP_LIB_PATH=$L/ab/w5.so
