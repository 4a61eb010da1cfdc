# Round 4: the shard-fallback diagnostic (stderr of the CLI under a 40 MB budget), the -m gpu files
# after test_shards_gpu's first failure, then the same-box A/B of gpu_r4_i.sh.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python tools/diag/shard_fallback.py > gpurun_out/r4j_diag.txt 2>&1 || { tail -20 gpurun_out/r4j_diag.txt; exit 1; }
cat gpurun_out/r4j_diag.txt
timeout -k 10 500 python -u -m pytest tests/test_shards_gpu.py tests/test_young_gpu.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4j_tests.log 2>&1; tail -4 gpurun_out/r4j_tests.log
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4j_$name.json 2> gpurun_out/r4j_$name.err || { tail -5 gpurun_out/r4j_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4j_$name.json
}
run r03 GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_r03/libgossip.so
run now
run r03_seq GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_r03/libgossip.so GOSSIP_YOUNG_OVERLAP=0
run now_seq GOSSIP_YOUNG_OVERLAP=0
