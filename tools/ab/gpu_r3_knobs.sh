# Round 3: C4 knob sweep after the DPP change, shard 0 of 2 only (--rehearse-shards 2: one
# shard-tick per step, the bench's N = 1 per-shard work), 20 timed ticks after 5 warm-up.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3k_$name.json 2> gpurun_out/r3k_$name.err || { tail -5 gpurun_out/r3k_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3k_$name.json
}
run base GOSSIP_X=0
run age4 GOSSIP_YOUNG_AGE=4
run age6 GOSSIP_YOUNG_AGE=6
run lpw64 GOSSIP_PULL_LPW=64
run lpw16 GOSSIP_PULL_LPW=16
run seq GOSSIP_YOUNG_OVERLAP=0
run grid8k GOSSIP_PULL_GRID=8192
