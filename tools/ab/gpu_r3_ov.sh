# Round 3: the two-stream pull phase after the register cuts: launch order / priority
# (young_overlap 1-4) and k_pull_young grid sizes, C4 shard 0 of 2.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3v_$name.json 2> gpurun_out/r3v_$name.err || { tail -5 gpurun_out/r3v_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3v_$name.json
}
run ov1 GOSSIP_YOUNG_OVERLAP=1
run ov2 GOSSIP_YOUNG_OVERLAP=2
run ov3 GOSSIP_YOUNG_OVERLAP=3
run ov4 GOSSIP_YOUNG_OVERLAP=4
run yg4k GOSSIP_YOUNG_GRID=4096
run yg2k GOSSIP_YOUNG_GRID=2048
run yg1k GOSSIP_YOUNG_GRID=1024
