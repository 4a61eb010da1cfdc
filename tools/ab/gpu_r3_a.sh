# Round 3, call A: the DENSE phase after k_dense_dedup (C2 hop-batched, C5 flood: bench + kernel
# trace), then the new / reshaped GPU tests (C3 at full size, C4 slice == continuous, trimmed
# oracle runs) with their durations.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for C in "c2 --batch" "c5 --width 4096"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -k 10 300 python tools/bench_dense.py $C --modes dense > gpurun_out/r3_dense_$tag.json 2> gpurun_out/r3_dense_$tag.err || { echo "bench $tag failed"; tail -5 gpurun_out/r3_dense_$tag.err; exit 1; }
  cat gpurun_out/r3_dense_$tag.json
done
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3_prof_c2 -o run --output-format csv -- python $R/tools/bench_dense.py c2 --batch --modes dense > $R/gpurun_out/r3_prof_c2.json 2> $R/gpurun_out/r3_prof_c2.err) || { echo "rocprof c2 failed"; exit 1; }
head -8 gpurun_out/r3_prof_c2/run_kernel_stats.csv
timeout -k 10 1000 python -u -m pytest tests/test_c3_gpu.py tests/test_scale_gpu.py tests/test_late_exit_gpu.py tests/test_row_partition.py tests/test_young_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread --durations=0 > gpurun_out/r3_tests_a.log 2>&1
rc=$?; tail -40 gpurun_out/r3_tests_a.log; exit $rc
