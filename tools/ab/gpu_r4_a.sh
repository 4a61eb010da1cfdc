# Round 4: saturation bits + dense-row tiles in k_pull -- the parity tests of the small paths,
# then the driver's bench command (C4, N = 1).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_young_gpu.py tests/test_late_exit_gpu.py > gpurun_out/r4a_tests.log 2>&1 || { tail -30 gpurun_out/r4a_tests.log; exit 1; }
tail -3 gpurun_out/r4a_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err || { tail -5 gpurun_out/r4a_bench.err; exit 1; }
python tools/ab_line.py sat_dr gpurun_out/r4a_bench.json
GOSSIP_PULL_SAT=0 GOSSIP_DENSE_ROWS=0 timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4a_bench_off.json 2> gpurun_out/r4a_bench_off.err || { tail -5 gpurun_out/r4a_bench_off.err; exit 1; }
python tools/ab_line.py off gpurun_out/r4a_bench_off.json
