# Round 3: C4 shard pull grid with the final kernels (non-temporal cap 16,384 blocks).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3g4_$name.json 2> gpurun_out/r3g4_$name.err || { tail -5 gpurun_out/r3g4_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3g4_$name.json
}
run g16k GOSSIP_X=0
run g8k GOSSIP_PULL_GRID=8192
run g32k GOSSIP_PULL_GRID=32768
run g16ky8k GOSSIP_YOUNG_GRID=8192
