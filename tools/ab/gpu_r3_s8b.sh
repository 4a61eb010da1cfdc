# Round 3: one rank of the 8-GPU C4 layout with the final kernels (young_nt on): young off (auto)
# vs forced on; the 4-GPU rank for the record.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, shards, env...
  local name=$1; local sh=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards $sh --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3b_$name.json 2> gpurun_out/r3b_$name.err || { tail -5 gpurun_out/r3b_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3b_$name.json
}
run s8auto 8 GOSSIP_X=0
run s8young1 8 GOSSIP_YOUNG=1
run s4auto 4 GOSSIP_X=0
run s2auto 2 GOSSIP_X=0
