# Round 6: k_pull_young split into its sparse-tick and dense-tick instantiations (lib/r6e): the C4
# N = 1 line against the round-5 library, the young tests, and the C4-scale tests of the 8-GPU
# layout's birth-tick rule (ORACLE A / ORACLE B / the continuous run).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
L=$R/p2p-gossip-simulation-ns3_amd/lib
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  GOSSIP_LIB_PATH=$L/$lib/libgossip.so timeout -k 10 500 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/r6g_$name.json 2> gpurun_out/r6g_$name.err || { tail -5 gpurun_out/r6g_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r6g_$name.json
}
run c4_r6e r6e --steps 20 --warmup 5
run c4_r5 r5 --steps 20 --warmup 5
run c4_r6e_2 r6e --steps 20 --warmup 5
timeout -k 10 400 python -u -m pytest tests/test_young_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r6g_young.log 2>&1 || { tail -30 gpurun_out/r6g_young.log; exit 1; }
tail -1 gpurun_out/r6g_young.log
timeout -k 10 900 python -u -m pytest tests/test_scale_gpu.py -k "c4" -x -v -m gpu --timeout 400 --timeout-method thread --durations=0 > gpurun_out/r6g_scale.log 2>&1 || { tail -40 gpurun_out/r6g_scale.log; exit 1; }
grep -E "passed|failed|PASSED|FAILED|s call" gpurun_out/r6g_scale.log | tail -12
