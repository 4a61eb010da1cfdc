# Round 4: seen lists in k_pull_young (+ saturation bits / dense rows in k_pull): parity of the
# small paths, the driver's bench command, the same with pull_sat / dense_rows off, and one SQ
# and two PMC passes over one C4 shard.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_young_gpu.py tests/test_engine_gpu.py tests/test_late_exit_gpu.py tests/test_row_partition.py > gpurun_out/r4b_tests.log 2>&1 || { tail -30 gpurun_out/r4b_tests.log; exit 1; }
tail -2 gpurun_out/r4b_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.err || { tail -5 gpurun_out/r4b_bench.err; exit 1; }
python tools/ab_line.py lists gpurun_out/r4b_bench.json
GOSSIP_PULL_SAT=0 GOSSIP_DENSE_ROWS=0 timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4b_bench_off.json 2> gpurun_out/r4b_bench_off.err || { tail -5 gpurun_out/r4b_bench_off.err; exit 1; }
python tools/ab_line.py lists_satoff gpurun_out/r4b_bench_off.json
GOSSIP_PULL_ROWS=0 timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4b_bench_norows.json 2> gpurun_out/r4b_bench_norows.err || { tail -5 gpurun_out/r4b_bench_norows.err; exit 1; }
python tools/ab_line.py norows gpurun_out/r4b_bench_norows.json
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --rehearse-shards 2 --steps 5 --warmup 5 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d $R/gpurun_out/r4b_sq -o run --output-format csv -- $B > $R/gpurun_out/r4b_sq.json 2> $R/gpurun_out/r4b_sq.err || { echo "sq failed"; tail -3 $R/gpurun_out/r4b_sq.err; exit 1; }
for k in "k_pull<32" "k_pull_rows" "k_pull_young"; do echo "$k"; python $R/tools/pmc_counters.py --timed 5 --kernel "$k" $R/gpurun_out/r4b_sq/run_counter_collection.csv; done
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r4b_pmcF -o run --output-format csv -- $B > $R/gpurun_out/r4b_pmcF.json 2> $R/gpurun_out/r4b_pmcF.err || { echo "pmcF failed"; tail -3 $R/gpurun_out/r4b_pmcF.err; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r4b_pmcW -o run --output-format csv -- $B > $R/gpurun_out/r4b_pmcW.json 2> $R/gpurun_out/r4b_pmcW.err || { echo "pmcW failed"; tail -3 $R/gpurun_out/r4b_pmcW.err; exit 1; }
for k in "k_pull<32" "k_pull_rows" "k_pull_young"; do echo "$k"; python $R/tools/pmc_counters.py --timed 5 --kernel "$k" $R/gpurun_out/r4b_pmcF/run_counter_collection.csv $R/gpurun_out/r4b_pmcW/run_counter_collection.csv; done
