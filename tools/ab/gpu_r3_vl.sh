# Round 3: a 3-peer first batch for passes of very late tiles (pull_vlate_age 7 / 8 / 9 vs off):
# parity subset with the option on, then the C4 shard A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
GOSSIP_PULL_VLATE_AGE=3 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_late_exit_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3vl_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3vl_tests.log; [ $rc -eq 0 ] || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3vl_$name.json 2> gpurun_out/r3vl_$name.err || { tail -5 gpurun_out/r3vl_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3vl_$name.json
}
run off GOSSIP_PULL_VLATE_AGE=0
run v7 GOSSIP_PULL_VLATE_AGE=7
run v8 GOSSIP_PULL_VLATE_AGE=8
run v9 GOSSIP_PULL_VLATE_AGE=9
