# Round 4: launch knobs on the final kernels (env-var engine options, one box): k_pull lanes per
# node 64 (8 tiles per pass), k_pull grid 8k / 32k blocks, k_pull_young grid 4k / 32k blocks.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4l_$name.json 2> gpurun_out/r4l_$name.err || { tail -5 gpurun_out/r4l_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4l_$name.json
}
run now
run lpw64 GOSSIP_PULL_LPW=64
run grid8k GOSSIP_PULL_GRID=8192
run grid32k GOSSIP_PULL_GRID=32768
run ygrid4k GOSSIP_YOUNG_GRID=4096
run ygrid32k GOSSIP_YOUNG_GRID=32768
