# Round 3: young-tile age on one rank of the 4- and 8-GPU C4 layouts (the auto rule keeps young
# off at 8 shards: ~12 expected slot entries per node at age 5).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, shards, env...
  local name=$1; local sh=$2; shift; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards $sh --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3a_$name.json 2> gpurun_out/r3a_$name.err || { tail -5 gpurun_out/r3a_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3a_$name.json
}
run s8off 8 GOSSIP_YOUNG=0
run s8a4 8 GOSSIP_YOUNG=1 GOSSIP_YOUNG_AGE=4
run s8a3 8 GOSSIP_YOUNG=1 GOSSIP_YOUNG_AGE=3
run s8a6 8 GOSSIP_YOUNG=1 GOSSIP_YOUNG_AGE=6
run s4a4 4 GOSSIP_YOUNG_AGE=4
run s4a6 4 GOSSIP_YOUNG_AGE=6
