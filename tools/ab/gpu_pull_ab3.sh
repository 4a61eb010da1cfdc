# A/B of k_pull's shape with the early exit on (round 2): k_pull alone vs concurrent with
# k_pull_young, peer loads in flight per lane (PULL_INFLIGHT 4 / 8 / 12 builds), grid size.
set -o pipefail
R=$GRAFT_REPO_ROOT
L=$R/p2p-gossip-simulation-ns3_amd/lib
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "$name failed"; tail -3 gpurun_out/ab_$name.err; exit 1; }
    python tools/ab_line.py $name gpurun_out/ab_$name.json
}
run seq GOSSIP_YOUNG_OVERLAP=0
run q12 GOSSIP_LIB_PATH=$L/libgossip_q12.so
run q4 GOSSIP_LIB_PATH=$L/libgossip_q4.so
run grid32k GOSSIP_PULL_GRID=32768
run grid8k GOSSIP_PULL_GRID=8192
