# PMC passes (separate runs, counters only): FETCH_SIZE and WRITE_SIZE for the default bench
# and for the dense-pull calibration run (--noskip, known algorithmic bytes).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_p.json 2>/dev/null && cat gpurun_out/bench_p.json || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --noskip > gpurun_out/bench_p_noskip.json 2>/dev/null && cat gpurun_out/bench_p_noskip.json || exit 1
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for mode in "" "--noskip"; do
  tag=skip; [ -n "$mode" ] && tag=noskip
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmcF_$tag -o run --output-format csv -- python $R/bench.py --no-cpu-baseline $mode > /dev/null 2>&1 || { echo "pmcF $tag failed"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmcW_$tag -o run --output-format csv -- python $R/bench.py --no-cpu-baseline $mode > /dev/null 2>&1 || { echo "pmcW $tag failed"; exit 1; }
done
echo pmc done
