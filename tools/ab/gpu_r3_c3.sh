# Round 3: C3 (1M nodes) pull grid and lanes per node with the final kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > gpurun_out/r3c3_$name.json 2> gpurun_out/r3c3_$name.err || { tail -5 gpurun_out/r3c3_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3c3_$name.json
}
run base GOSSIP_X=0
run g1k GOSSIP_PULL_GRID=1024
run g4k GOSSIP_PULL_GRID=4096
run g8k GOSSIP_PULL_GRID=8192
run lpw16 GOSSIP_PULL_LPW=16
run nt1 GOSSIP_PULL_NT=1
