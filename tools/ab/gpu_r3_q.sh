# Round 3: k_pull without the dead incoming-word path (88 VGPRs at 6 loads in flight): parity
# subset, then C4 shard A/B of 5 / 6 / 7 / 8 loads in flight (all at 5 waves per SIMD).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_late_exit_gpu.py tests/test_hop_batch.py "tests/test_scale_gpu.py::test_c4_sample_matches_oracle_a" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3q_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3q_tests.log; [ $rc -eq 0 ] || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3q_$name.json 2> gpurun_out/r3q_$name.err || { tail -5 gpurun_out/r3q_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3q_$name.json
}
L=$R/p2p-gossip-simulation-ns3_amd/lib
run q6 GOSSIP_X=0
run q5 GOSSIP_LIB_PATH=$L/ab/q5.so
run q7 GOSSIP_LIB_PATH=$L/ab/q7.so
run q8 GOSSIP_LIB_PATH=$L/ab/q8.so
run q6seq GOSSIP_YOUNG_OVERLAP=0
