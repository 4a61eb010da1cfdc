# Round 5: k_dense_fused's tail fills the blocks' deficits below the mean load: parity, then a
# same-box A/B of the C2 / C5 lines -- this build, its rounds capped (GOSSIP_DENSE_ROUNDS = 0: pure
# stream-K; 1), the previous build (lib/var_r5f) -- and the DENSE_STAMPS build.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_dense_fused_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/r5h_fused_tests.log 2>&1 || { tail -40 gpurun_out/r5h_fused_tests.log; exit 1; }
tail -1 gpurun_out/r5h_fused_tests.log
timeout -k 10 900 python -u -m pytest tests/test_hop_batch.py tests/test_scale_gpu.py -k "c2 or c5 or hop_batch" -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r5h_dense_tests.log 2>&1 || { tail -40 gpurun_out/r5h_dense_tests.log; exit 1; }
tail -1 gpurun_out/r5h_dense_tests.log
L=$R/p2p-gossip-simulation-ns3_amd/lib
one() {  # name, env..., then the bench_dense args after --
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 400 python tools/bench_dense.py "$@" --modes dense > gpurun_out/r5h_$name.json 2> gpurun_out/r5h_$name.err || { tail -5 gpurun_out/r5h_$name.err; exit 1; }
  python tools/ab_dense.py $name gpurun_out/r5h_$name.json
}
for rep in 1 2; do
  for c in c2 c5; do
    a="$c"; [ $c = c2 ] && a="c2 --batch"
    one ${c}_cur$rep X=1 -- $a
    one ${c}_r0_$rep GOSSIP_DENSE_ROUNDS=0 -- $a
    one ${c}_r1_$rep GOSSIP_DENSE_ROUNDS=1 -- $a
    one ${c}_prev$rep GOSSIP_LIB_PATH=$L/var_r5f/libgossip.so -- $a
  done
done
one c2_ds GOSSIP_LIB_PATH=$L/diag_ds/libgossip.so -- c2 --batch
grep dense_stamps gpurun_out/r5h_c2_ds.err | tail -1
