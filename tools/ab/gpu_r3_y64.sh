# Round 3: k_pull_young at 64 VGPRs (explicit-lane shuffles, no hoisted lane values): young parity
# + C4 ORACLE A sample, then the C4 shard bench (concurrent and in sequence).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_young_gpu.py tests/test_late_exit_gpu.py "tests/test_scale_gpu.py::test_c4_sample_matches_oracle_a" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3y_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3y_tests.log; [ $rc -eq 0 ] || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3y_$name.json 2> gpurun_out/r3y_$name.err || { tail -5 gpurun_out/r3y_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3y_$name.json
}
run y64 GOSSIP_X=0
run y64seq GOSSIP_YOUNG_OVERLAP=0
run y64own GOSSIP_YOUNG_OWN=1 GOSSIP_YOUNG_OVERLAP=0
