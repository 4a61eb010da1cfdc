# quick GPU iteration: parity tests, one bench line, rocprof kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/gpu_tests.log | tail -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { echo bench failed; tail gpurun_out/bench_q.err; exit 1; }
cat gpurun_out/bench_q.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_q -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench_q_prof.json 2>/dev/null || { echo prof failed; exit 1; }
head -4 $GRAFT_REPO_ROOT/gpurun_out/prof_q/run_kernel_stats.csv | cut -c1-160
