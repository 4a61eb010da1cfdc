# Round 3: age-ordered tile lists (pull_tile_order) + young_own tests; C4 shard A/B in one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_young_gpu.py tests/test_late_exit_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3r_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3r_tests.log; [ $rc -eq 0 ] || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3r_$name.json 2> gpurun_out/r3r_$name.err || { tail -5 gpurun_out/r3r_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3r_$name.json
}
run order1 GOSSIP_PULL_TILE_ORDER=1
run order0 GOSSIP_PULL_TILE_ORDER=0
run order1seq GOSSIP_PULL_TILE_ORDER=1 GOSSIP_YOUNG_OVERLAP=0
run order0seq GOSSIP_PULL_TILE_ORDER=0 GOSSIP_YOUNG_OVERLAP=0
