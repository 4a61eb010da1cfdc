# Round 4: k_pull gathers with one lane shuffle per peer (id and tile bits packed):
# parity (engine, young, late-exit, C4 headline vs ORACLE B, C4 and C3 slice vs continuous),
# then the same-box A/B against the previous build (lib/ab_prev), concurrent and alone.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py tests/test_late_exit_gpu.py "tests/test_scale_gpu.py::test_c4_headline_kernels_match_oracle_b" -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4o_tests.log 2>&1 || { tail -30 gpurun_out/r4o_tests.log; exit 1; }
tail -3 gpurun_out/r4o_tests.log
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4o_$name.json 2> gpurun_out/r4o_$name.err || { tail -5 gpurun_out/r4o_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4o_$name.json
}
run prev GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_prev/libgossip.so
run now
run prev_seq GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_prev/libgossip.so GOSSIP_YOUNG_OVERLAP=0
run now_seq GOSSIP_YOUNG_OVERLAP=0
