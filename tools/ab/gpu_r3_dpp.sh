# Round 3: k_pull with DPP group reductions and the node's peer range read once per node:
# parity first, then the C4 bench (concurrent, and in sequence for each kernel's own time).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_young_gpu.py tests/test_late_exit_gpu.py tests/test_hop_batch.py tests/test_row_partition.py tests/test_c3_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r3p_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3p_bench.json 2> gpurun_out/r3p_bench.err || { tail -5 gpurun_out/r3p_bench.err; exit 1; }
python tools/ab_line.py dpp gpurun_out/r3p_bench.json
GOSSIP_YOUNG_OVERLAP=0 timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3p_bench_seq.json 2> gpurun_out/r3p_bench_seq.err || { tail -5 gpurun_out/r3p_bench_seq.err; exit 1; }
python tools/ab_line.py dpp_seq gpurun_out/r3p_bench_seq.json
