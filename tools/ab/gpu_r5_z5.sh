# Round 5: one rank of 8 shards at the new default (tick rule, fresh tile per birth tick): young_age
# 4 / 6, dense rows off, young grid 64k, between two default runs, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 > gpurun_out/r5z5_$name.json 2> gpurun_out/r5z5_$name.err || { tail -5 gpurun_out/r5z5_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r5z5_$name.json
}
run auto1 X=1
run age4 GOSSIP_YOUNG_AGE=4
run age6 GOSSIP_YOUNG_AGE=6
run dr0 GOSSIP_DENSE_ROWS=0
run ygrid64k GOSSIP_YOUNG_GRID=65536
run auto2 X=1
