# Round 5: k_dense_fused's grouped tile order (GM row blocks x column tiles per group): parity,
# then a same-box A/B of the C2 / C5 lines over GOSSIP_DENSE_GM = 1 (row-major, the previous
# order), 4, 8 (default), 16; then tools/ab/gpu_r5_i.sh (k_pull_young segment counts).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_dense_fused_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/r5j_fused_tests.log 2>&1 || { tail -40 gpurun_out/r5j_fused_tests.log; exit 1; }
tail -1 gpurun_out/r5j_fused_tests.log
timeout -k 10 900 python -u -m pytest tests/test_hop_batch.py tests/test_scale_gpu.py -k "c2 or c5 or hop_batch" -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r5j_dense_tests.log 2>&1 || { tail -40 gpurun_out/r5j_dense_tests.log; exit 1; }
tail -1 gpurun_out/r5j_dense_tests.log
one() {  # name, env..., then the bench_dense args after --
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 400 python tools/bench_dense.py "$@" --modes dense > gpurun_out/r5j_$name.json 2> gpurun_out/r5j_$name.err || { tail -5 gpurun_out/r5j_$name.err; exit 1; }
  python tools/ab_dense.py $name gpurun_out/r5j_$name.json
}
for rep in 1 2; do
  for c in c2 c5; do
    a="$c"; [ $c = c2 ] && a="c2 --batch"
    for gm in 1 4 8 16; do one ${c}_gm${gm}_$rep GOSSIP_DENSE_GM=$gm -- $a; done
  done
done
bash tools/ab/gpu_r5_i.sh
