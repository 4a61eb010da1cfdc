# Round 4: k_pull_young with one fused per-tile pass (no touched-word list), DPP scans; parity, then A/B vs r03 and an 8-wave build.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_young_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4f_tests.log 2>&1 || { tail -30 gpurun_out/r4f_tests.log; exit 1; }
tail -3 gpurun_out/r4f_tests.log
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4f_$name.json 2> gpurun_out/r4f_$name.err || { tail -5 gpurun_out/r4f_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4f_$name.json
}
run r03 GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_r03/libgossip.so
run now
run r03_seq GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_r03/libgossip.so GOSSIP_YOUNG_OVERLAP=0
run now_seq GOSSIP_YOUNG_OVERLAP=0
run y8_seq GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_y8/libgossip.so GOSSIP_YOUNG_OVERLAP=0
run y8 GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_y8/libgossip.so
