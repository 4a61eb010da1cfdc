# Round 5: one rank of the 8-GPU C4 layout (birth-tick rule): k_pull's skipping options by
# environment, same box -- dense-row tiles off, early exit off / from age 2, saturation bits off,
# seen gate off, tile lists in tile order -- between two default runs.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 > gpurun_out/r5v_$name.json 2> gpurun_out/r5v_$name.err || { tail -5 gpurun_out/r5v_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r5v_$name.json
}
run auto1 X=1
run dr0 GOSSIP_DENSE_ROWS=0
run dr1 GOSSIP_DENSE_ROWS=1
run late0 GOSSIP_LATE_AGE=0
run late2 GOSSIP_LATE_AGE=2
run sat0 GOSSIP_PULL_SAT=0
run gate0 GOSSIP_PULL_GATE=0
run order0 GOSSIP_PULL_TILE_ORDER=0
run auto2 X=1
