# A/B of the bottom-up early exit in k_pull on C4 (driver command shape): k_pull alone
# (young_overlap 0) and the concurrent phase, base vs libgossip_ee.so.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 400 $B > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "$name failed"; tail -3 gpurun_out/ab_$name.err; exit 1; }
    python tools/ab_line.py $name gpurun_out/ab_$name.json
}
run base_seq GOSSIP_YOUNG_OVERLAP=0
run ee_seq GOSSIP_YOUNG_OVERLAP=0 GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/libgossip_ee.so
run ee_overlap GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/libgossip_ee.so
