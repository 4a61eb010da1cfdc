# rocprofv3 evidence for the C4 bench line: kernel trace + stats of the default command, then
# one PMC pass per counter (FETCH_SIZE, WRITE_SIZE) for the HBM traffic of k_pull.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c4 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/c4_bench_prof.json 2> $R/gpurun_out/c4_bench_prof.err || { echo "kernel trace failed"; tail -5 $R/gpurun_out/c4_bench_prof.err; exit 1; }
timeout -s KILL 420 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmcF4 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > /dev/null 2> $R/gpurun_out/pmcF4.err || { echo "FETCH_SIZE pass failed"; tail -3 $R/gpurun_out/pmcF4.err; exit 1; }
timeout -s KILL 420 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmcW4 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > /dev/null 2> $R/gpurun_out/pmcW4.err || { echo "WRITE_SIZE pass failed"; tail -3 $R/gpurun_out/pmcW4.err; exit 1; }
cd $R
python3 tools/prof_summary.py gpurun_out/prof_c4 run --timed 40 --passes 2 --out gpurun_out/c4_summary.json > /dev/null && python3 tools/pmc_traffic.py gpurun_out/pmcF4/run_counter_collection.csv gpurun_out/pmcW4/run_counter_collection.csv --timed 40 --passes 2 --out gpurun_out/pmc_C4.json && head -c 1500 gpurun_out/c4_summary.json && cat gpurun_out/c4_bench_prof.json
