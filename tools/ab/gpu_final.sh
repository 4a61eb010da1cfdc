# Round evidence: GPU parity suite, the default bench line (with the CPU baseline), then the
# rocprofv3 kernel trace and the two PMC passes of tools/gpu_prof_c4.sh.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { echo "bench failed"; tail -3 gpurun_out/bench_final.err; exit 1; }
cat gpurun_out/bench_final.json
bash tools/gpu_prof_c4.sh
