# Round 3: one rank of the 8-GPU C4 layout (shard 0 of 8): pull grid and non-temporal rows.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3s8g_$name.json 2> gpurun_out/r3s8g_$name.err || { tail -5 gpurun_out/r3s8g_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3s8g_$name.json
}
run base GOSSIP_X=0
run g8k GOSSIP_PULL_GRID=8192
run g32k GOSSIP_PULL_GRID=32768
run nt0 GOSSIP_PULL_NT=0
run nt0g4k GOSSIP_PULL_NT=0 GOSSIP_PULL_GRID=4096
