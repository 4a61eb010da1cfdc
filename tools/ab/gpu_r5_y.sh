# Round 5: a fresh tile per birth tick (GOSSIP_F_TILE_PER_TICK: no tile mixes two ticks' births)
# on one rank of 8 shards (birth-tick rule) and on the C4 line, against the default, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env, bench args...
  local name=$1 envs=$2; shift 2
  env $envs timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/r5y_$name.json 2> gpurun_out/r5y_$name.err || { tail -5 gpurun_out/r5y_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r5y_$name.json
}
run s8_base X=1 --rehearse-shards 8
run s8_tpt GOSSIP_BENCH_TILE_PER_TICK=1 --rehearse-shards 8
run s8_base2 X=1 --rehearse-shards 8
run s8_tpt2 GOSSIP_BENCH_TILE_PER_TICK=1 --rehearse-shards 8
run s4_tpt GOSSIP_BENCH_TILE_PER_TICK=1 --rehearse-shards 4
run c4_base X=1
run c4_tpt GOSSIP_BENCH_TILE_PER_TICK=1
