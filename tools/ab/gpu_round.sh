set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?"; grep -E "passed|failed" gpurun_out/gpu_tests.log | tail -3
timeout -k 10 300 python bench.py > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { echo bench failed; tail gpurun_out/bench2.err; exit 1; }
cat gpurun_out/bench2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof2 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/bench2_prof.json 2>/dev/null || { echo prof failed; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/pmcF -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > /dev/null 2>$GRAFT_REPO_ROOT/gpurun_out/pmcF.err || { echo pmcF failed; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/pmcW -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline > /dev/null 2>$GRAFT_REPO_ROOT/gpurun_out/pmcW.err || { echo pmcW failed; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --gpus 4 --rehearse-shards 4 --no-cpu-baseline --steps 10 --warmup 20 > gpurun_out/rehearse4.json 2> gpurun_out/rehearse4.err; echo "rehearse4 rc=$?"; cat gpurun_out/rehearse4.json; tail -2 gpurun_out/rehearse4.err
