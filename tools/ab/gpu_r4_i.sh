# Round 4: sent derived from recv (births' sends + deg x recv; the pull kernels load no |peers|),
# k_pull's explicit wait before its stores, k_pull_young's single dedup pass: the whole -m gpu
# suite, then the same-box A/B against r03 (kernels alone and concurrent) and the stamp build.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4i_tests.log 2>&1 || { tail -30 gpurun_out/r4i_tests.log; exit 1; }
tail -3 gpurun_out/r4i_tests.log
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4i_$name.json 2> gpurun_out/r4i_$name.err || { tail -5 gpurun_out/r4i_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4i_$name.json
}
run r03 GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_r03/libgossip.so
run now
run r03_seq GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_r03/libgossip.so GOSSIP_YOUNG_OVERLAP=0
run now_seq GOSSIP_YOUNG_OVERLAP=0
run ys_seq GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_ys/libgossip.so GOSSIP_YOUNG_OVERLAP=0
grep young_stamps gpurun_out/r4i_ys_seq.err | tail -2
