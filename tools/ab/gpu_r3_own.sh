# Round 3: k_pull_young own-frontier dedup (option young_own): young parity suite + C4 sample vs
# ORACLE A + C4 slice-vs-continuous, then the C4 per-shard A/B (young_own 1 / 0).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_young_gpu.py tests/test_late_exit_gpu.py tests/test_engine_gpu.py tests/test_c3_gpu.py "tests/test_scale_gpu.py::test_c4_sample_matches_oracle_a" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3o_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r3o_tests.log; [ $rc -eq 0 ] || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3o_$name.json 2> gpurun_out/r3o_$name.err || { tail -5 gpurun_out/r3o_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3o_$name.json
}
run own1 GOSSIP_YOUNG_OWN=1
run own0 GOSSIP_YOUNG_OWN=0
run own1seq GOSSIP_YOUNG_OWN=1 GOSSIP_YOUNG_OVERLAP=0
