# Round 4: k_pull_young grids above 32k blocks (64k .. 2^20), the driver's bench arguments, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4u_$name.json 2> gpurun_out/r4u_$name.err || { tail -5 gpurun_out/r4u_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4u_$name.json
}
run y64k GOSSIP_YOUNG_GRID=65536
run y128k GOSSIP_YOUNG_GRID=131072
run y256k GOSSIP_YOUNG_GRID=262144
run y1m GOSSIP_YOUNG_GRID=1048576
run y64k_2 GOSSIP_YOUNG_GRID=65536
run y128k_2 GOSSIP_YOUNG_GRID=131072
