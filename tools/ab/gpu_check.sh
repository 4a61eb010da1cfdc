# round re-entry check: full GPU parity suite, default bench (with CPU baseline), N=2 rehearsal
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" gpurun_out/gpu_tests.log | tail -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err || { echo bench failed; tail gpurun_out/bench_c.err; exit 1; }
cat gpurun_out/bench_c.json
timeout -k 10 400 python bench.py --gpus 2 --rehearse-shards 2 --no-cpu-baseline --steps 10 --warmup 20 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err; echo "rehearse2 rc=$?"; cat gpurun_out/rehearse2.json; tail -3 gpurun_out/rehearse2.err
