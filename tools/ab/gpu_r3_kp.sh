# Round 3: k_pull with explicit-lane shuffles and `want` carried past the gather (125 -> 100
# VGPRs): parity, then C4 shard A/B against 6 loads in flight (93 VGPRs, 5 waves/SIMD) and a
# 5-wave register cap on 8 loads.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_young_gpu.py tests/test_late_exit_gpu.py tests/test_c3_gpu.py "tests/test_scale_gpu.py::test_c4_sample_matches_oracle_a" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3p2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3p2_tests.log; [ $rc -eq 0 ] || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3p2_$name.json 2> gpurun_out/r3p2_$name.err || { tail -5 gpurun_out/r3p2_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3p2_$name.json
}
L=$R/p2p-gossip-simulation-ns3_amd/lib
run q8 GOSSIP_X=0
run q6 GOSSIP_LIB_PATH=$L/ab/q6.so
run q8w5 GOSSIP_LIB_PATH=$L/ab/w5.so
run q8seq GOSSIP_YOUNG_OVERLAP=0
run q6seq GOSSIP_YOUNG_OVERLAP=0 GOSSIP_LIB_PATH=$L/ab/q6.so
