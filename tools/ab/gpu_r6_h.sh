# Round 6: C5's row ranks through k_dense_fused with the FT slice exchange (lib/r6f): the row-partition
# and fused-dense tests, the C5 row-partition test of 2 and 8 ranks, then tools/bench_dense.py c5
# --row-shards 8 (per-rank phase, exchange bytes) and the single-GPU C5 / C2 lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_row_partition.py tests/test_dense_fused_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r6h_tests.log 2>&1 || { tail -30 gpurun_out/r6h_tests.log; exit 1; }
tail -1 gpurun_out/r6h_tests.log
timeout -k 10 600 python -u -m pytest tests/test_scale_gpu.py -k "c5_row" -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6h_c5rows.log 2>&1 || { tail -30 gpurun_out/r6h_c5rows.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r6h_c5rows.log | tail -3
timeout -k 10 300 python -u tools/bench_dense.py c5 --row-shards 8 > gpurun_out/r6h_c5_rows8.json 2> gpurun_out/r6h_c5_rows8.err || { tail -5 gpurun_out/r6h_c5_rows8.err; exit 1; }
tail -c 1500 gpurun_out/r6h_c5_rows8.json
