# Round 4: same-box A/B of the round-3 engine (lib/ab_r03, built from commit b9d8daa) and this
# tree, each with the two pull kernels concurrent (the default) and in sequence (each alone).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4d_$name.json 2> gpurun_out/r4d_$name.err || { tail -5 gpurun_out/r4d_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4d_$name.json
}
run r03 GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_r03/libgossip.so
run now GOSSIP_PULL_ROWS=0
run r03_seq GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_r03/libgossip.so GOSSIP_YOUNG_OVERLAP=0
run now_seq GOSSIP_YOUNG_OVERLAP=0
run now_seq_satoff GOSSIP_YOUNG_OVERLAP=0 GOSSIP_PULL_SAT=0 GOSSIP_DENSE_ROWS=0
