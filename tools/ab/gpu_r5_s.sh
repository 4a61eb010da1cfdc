# Round 5: one rank of the 8-GPU C4 layout (birth-tick rule, bench's auto at 8 shards): launch
# shapes by engine option, same box -- pull grid 8k / 32k blocks, young grid 16k / 64k, cached
# (not non-temporal) pull rows and young slot lines -- between two default runs.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 > gpurun_out/r5s_$name.json 2> gpurun_out/r5s_$name.err || { tail -5 gpurun_out/r5s_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r5s_$name.json
}
run auto1 X=1
run pgrid8k GOSSIP_PULL_GRID=8192
run pgrid32k GOSSIP_PULL_GRID=32768
run ygrid16k GOSSIP_YOUNG_GRID=16384
run ygrid64k GOSSIP_YOUNG_GRID=65536
run pnt0 GOSSIP_PULL_NT=0
run ynt0 GOSSIP_YOUNG_NT=0
run auto2 X=1
