# Round 6: the dense split-tile reduction without the release/acquire fences (each wave waits for its
# atomics' acknowledgements before the ticket) -- parity of the fused tests, then the C2 / C5 lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_dense_fused_gpu.py tests/test_row_partition.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r6j_tests.log 2>&1 || { tail -30 gpurun_out/r6j_tests.log; exit 1; }
tail -3 gpurun_out/r6j_tests.log
for c in c2 c5; do
  a="$c"; [ $c = c2 ] && a="c2 --batch"
  timeout -k 10 400 python tools/bench_dense.py $a --modes dense > gpurun_out/r6j_$c.json 2> gpurun_out/r6j_$c.err || { tail -5 gpurun_out/r6j_$c.err; exit 1; }
  python tools/ab_dense.py $c gpurun_out/r6j_$c.json
done
