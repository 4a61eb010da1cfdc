# Round 3: k_pull without the exit test before the first peer batch (ab/skip.so) vs the committed
# build, C4 shard, concurrent and k_pull alone.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3k2_$name.json 2> gpurun_out/r3k2_$name.err || { tail -5 gpurun_out/r3k2_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3k2_$name.json
}
L=$R/p2p-gossip-simulation-ns3_amd/lib
run base GOSSIP_X=0
run skip GOSSIP_LIB_PATH=$L/ab/skip.so
run baseseq GOSSIP_YOUNG_OVERLAP=0
run skipseq GOSSIP_YOUNG_OVERLAP=0 GOSSIP_LIB_PATH=$L/ab/skip.so
