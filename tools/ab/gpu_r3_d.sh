# Round 3, call D: row-partition tests after the capacity bound; the DENSE phase kernel trace
# after the replicated counters (C2 hop-batched); the C3 line (young on/off, trace, PMC).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_row_partition.py tests/test_multiprocess_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3d_rows_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3d_rows_tests.log; [ $rc -eq 0 ] || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3d_prof_c2 -o run --output-format csv -- python $R/tools/bench_dense.py c2 --batch --modes dense > $R/gpurun_out/r3d_prof_c2.json 2> $R/gpurun_out/r3d_prof_c2.err) || { echo "rocprof c2 failed"; exit 1; }
head -6 gpurun_out/r3d_prof_c2/run_kernel_stats.csv
bash tools/ab/gpu_prof_c3.sh
