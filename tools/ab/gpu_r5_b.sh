# Round 5: the fused DENSE kernel (k_dense_fused) -- parity first (fused vs three-kernel vs ORACLE
# A / B), then the C2 hop-batched and C5 (4,096 shares) lines and their rocprofv3 traces.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_dense_fused_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r5b_fused_tests.log 2>&1 || { tail -40 gpurun_out/r5b_fused_tests.log; exit 1; }
tail -3 gpurun_out/r5b_fused_tests.log
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k "dense_mfma or sharded_engines" tests/test_hop_batch.py tests/test_shards_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5b_dense_tests.log 2>&1 || { tail -40 gpurun_out/r5b_dense_tests.log; exit 1; }
tail -2 gpurun_out/r5b_dense_tests.log
timeout -k 10 300 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/r5b_c2.json 2> gpurun_out/r5b_c2.err || { tail -5 gpurun_out/r5b_c2.err; exit 1; }
cat gpurun_out/r5b_c2.json
timeout -k 10 400 python tools/bench_dense.py c5 --modes dense > gpurun_out/r5b_c5.json 2> gpurun_out/r5b_c5.err || { tail -5 gpurun_out/r5b_c5.err; exit 1; }
cat gpurun_out/r5b_c5.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5b_c2trace -o run --output-format csv -- python $R/tools/bench_dense.py c2 --batch --modes dense > $R/gpurun_out/r5b_c2trace.json 2> $R/gpurun_out/r5b_c2trace.err || { echo "c2 trace failed"; tail -3 $R/gpurun_out/r5b_c2trace.err; exit 1; }
echo c2 trace ok
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5b_c5trace -o run --output-format csv -- python $R/tools/bench_dense.py c5 --modes dense > $R/gpurun_out/r5b_c5trace.json 2> $R/gpurun_out/r5b_c5trace.err || { echo "c5 trace failed"; tail -3 $R/gpurun_out/r5b_c5trace.err; exit 1; }
echo c5 trace ok
