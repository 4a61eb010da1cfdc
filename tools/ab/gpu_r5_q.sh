# Round 5: one rank of the 8-GPU C4 layout under the birth-tick rule (bench's auto rule at 8 shards),
# young tiles auto / off / young_age 3 / 4 (first call), auto / young_age 6 / 7 (second) -- engine
# options by environment, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 > gpurun_out/r5q_$name.json 2> gpurun_out/r5q_$name.err || { tail -5 gpurun_out/r5q_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r5q_$name.json
}
run auto X=1
run age6 GOSSIP_YOUNG_AGE=6
run age7 GOSSIP_YOUNG_AGE=7



