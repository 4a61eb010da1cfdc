# Round 3: k_pull pass -> tile lists (option pull_tiles): parity suite first, then the C4 bench
# A/B (GOSSIP_PULL_TILES=0 / 1) and the DENSE phase timer.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_young_gpu.py tests/test_late_exit_gpu.py tests/test_hop_batch.py tests/test_row_partition.py tests/test_handshake.py tests/test_link_timing.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3t_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3t_tests.log; [ $rc -eq 0 ] || exit 1
for v in 1 0; do
  GOSSIP_PULL_TILES=$v timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3t_bench_t$v.json 2> gpurun_out/r3t_bench_t$v.err || { tail -5 gpurun_out/r3t_bench_t$v.err; exit 1; }
  python tools/ab_line.py tiles$v gpurun_out/r3t_bench_t$v.json
done
timeout -k 10 300 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/r3t_dense_c2.json 2> gpurun_out/r3t_dense_c2.err || exit 1
cat gpurun_out/r3t_dense_c2.json
