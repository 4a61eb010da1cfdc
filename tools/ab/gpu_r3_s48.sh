# Round 3: one rank of the 4- and 8-GPU C4 layouts (--rehearse-shards 4 / 8) with the round-3
# kernels: young tiles auto vs forced on/off (the auto rule's threshold was measured on r02 kernels).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, shards, env...
  local name=$1; local sh=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards $sh --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3s_$name.json 2> gpurun_out/r3s_$name.err || { tail -5 gpurun_out/r3s_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3s_$name.json
}
run s8auto 8 GOSSIP_X=0
run s8young1 8 GOSSIP_YOUNG=1
run s4auto 4 GOSSIP_X=0
run s4young0 4 GOSSIP_YOUNG=0
