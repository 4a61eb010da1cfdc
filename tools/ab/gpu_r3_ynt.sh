# Round 3: non-temporal slot-line loads in k_pull_young (young_nt 0 / 1), C4 shard, concurrent
# and in sequence.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3n_$name.json 2> gpurun_out/r3n_$name.err || { tail -5 gpurun_out/r3n_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3n_$name.json
}
run nt0 GOSSIP_YOUNG_NT=0
run nt1 GOSSIP_YOUNG_NT=1
run nt0seq GOSSIP_YOUNG_NT=0 GOSSIP_YOUNG_OVERLAP=0
run nt1seq GOSSIP_YOUNG_NT=1 GOSSIP_YOUNG_OVERLAP=0
