# Round 3, call C: replicated traffic counters (acct) -- the DENSE phase (C2 hop-batched, C5) and
# the C4 headline bench; dense parity tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for C in "c2 --batch" "c5 --width 4096"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -k 10 300 python tools/bench_dense.py $C --modes dense > gpurun_out/r3c_dense_$tag.json 2> gpurun_out/r3c_dense_$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/r3c_dense_$tag.err; exit 1; }
  cat gpurun_out/r3c_dense_$tag.json
done
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_hop_batch.py -m gpu -x -q --timeout 300 --timeout-method thread -k "dense or mfma or hop" > gpurun_out/r3c_dense_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3c_dense_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err || { tail -5 gpurun_out/r3c_bench.err; exit 1; }
python tools/ab_line.py c4 gpurun_out/r3c_bench.json
timeout -k 10 600 python -u -m pytest tests/test_row_partition.py tests/test_multiprocess_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3c_rows_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3c_rows_tests.log; [ $rc -eq 0 ] || exit 1
