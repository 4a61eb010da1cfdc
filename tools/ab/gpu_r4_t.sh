# Round 4: k_pull_young grid default 2x the pull grid (32,768 blocks at C4) against 16k and 64k,
# the driver's bench arguments, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4t_$name.json 2> gpurun_out/r4t_$name.err || { tail -5 gpurun_out/r4t_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4t_$name.json
}
run now
run y16k GOSSIP_YOUNG_GRID=16384
run y64k GOSSIP_YOUNG_GRID=65536
run now2
run y16k_2 GOSSIP_YOUNG_GRID=16384
