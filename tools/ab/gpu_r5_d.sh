# Round 5: the stream-K fused DENSE kernel -- parity (fused vs three-kernel vs ORACLE A / B, the
# C2 full run, C5 x 4,096 shares), then the C2 / C5 lines and rocprofv3 traces.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_dense_fused_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/r5d_fused_tests.log 2>&1 || { tail -40 gpurun_out/r5d_fused_tests.log; exit 1; }
tail -1 gpurun_out/r5d_fused_tests.log
timeout -k 10 900 python -u -m pytest tests/test_hop_batch.py tests/test_scale_gpu.py -k "c2 or c5 or hop_batch" tests/test_engine_gpu.py::test_dense_mfma_mode_matches_oracle -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/r5d_dense_tests.log 2>&1 || { tail -40 gpurun_out/r5d_dense_tests.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/r5d_dense_tests.log | tail -12
timeout -k 10 300 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/r5d_c2.json 2> gpurun_out/r5d_c2.err || { tail -5 gpurun_out/r5d_c2.err; exit 1; }
cat gpurun_out/r5d_c2.json
timeout -k 10 400 python tools/bench_dense.py c5 --modes dense > gpurun_out/r5d_c5.json 2> gpurun_out/r5d_c5.err || { tail -5 gpurun_out/r5d_c5.err; exit 1; }
cat gpurun_out/r5d_c5.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5d_c2trace -o run --output-format csv -- python $R/tools/bench_dense.py c2 --batch --modes dense > $R/gpurun_out/r5d_c2trace.json 2> $R/gpurun_out/r5d_c2trace.err || { echo "c2 trace failed"; tail -3 $R/gpurun_out/r5d_c2trace.err; exit 1; }
echo c2 trace ok
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5d_c5trace -o run --output-format csv -- python $R/tools/bench_dense.py c5 --modes dense > $R/gpurun_out/r5d_c5trace.json 2> $R/gpurun_out/r5d_c5trace.err || { echo "c5 trace failed"; tail -3 $R/gpurun_out/r5d_c5trace.err; exit 1; }
echo c5 trace ok
