# Round 4: k_pull_young variants on one box: A = unused peer groups not issued + slot headers by
# lead-lane ballots (71 VGPRs), B = header ballots only (67 VGPRs), against the final tree (64).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4q_$name.json 2> gpurun_out/r4q_$name.err || { tail -5 gpurun_out/r4q_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4q_$name.json
}
L=$R/p2p-gossip-simulation-ns3_amd/lib
run now
run a GOSSIP_LIB_PATH=$L/ab_a/libgossip.so
run b GOSSIP_LIB_PATH=$L/ab_b/libgossip.so
run now_seq GOSSIP_YOUNG_OVERLAP=0
run a_seq GOSSIP_LIB_PATH=$L/ab_a/libgossip.so GOSSIP_YOUNG_OVERLAP=0
run b_seq GOSSIP_LIB_PATH=$L/ab_b/libgossip.so GOSSIP_YOUNG_OVERLAP=0
run now2
