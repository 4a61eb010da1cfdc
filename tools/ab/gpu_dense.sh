# dense-mode iteration: dense parity tests, then C2 and the C5 slice (csr vs dense)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "dense or golden or hand" > gpurun_out/gpu_dense.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_dense.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/bench_dense.py c2 --modes dense > gpurun_out/dense_c2.json 2> gpurun_out/dense_c2.err || { echo c2 failed; tail gpurun_out/dense_c2.err; exit 1; }
cat gpurun_out/dense_c2.json
timeout -k 10 300 python -u tools/bench_dense.py c5 --width ${C5W:-1024} --modes ${C5M:-csr,dense} > gpurun_out/dense_c5.json 2> gpurun_out/dense_c5.err || { echo c5 failed; tail gpurun_out/dense_c5.err; exit 1; }
cat gpurun_out/dense_c5.json
