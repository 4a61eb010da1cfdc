# Round 3: PMC HBM traffic of the pull kernels under the driver's bench command (one pass per
# counter; the profiler serialises the kernels), converted by tools/pmc_traffic.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
timeout -s KILL 450 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r3_pmcF -o run --output-format csv -- $B > $R/gpurun_out/r3_pmcF.json 2> $R/gpurun_out/r3_pmcF.err || { echo "pmcF failed"; tail -3 $R/gpurun_out/r3_pmcF.err; exit 1; }
echo pmcF ok
timeout -s KILL 450 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r3_pmcW -o run --output-format csv -- $B > $R/gpurun_out/r3_pmcW.json 2> $R/gpurun_out/r3_pmcW.err || { echo "pmcW failed"; tail -3 $R/gpurun_out/r3_pmcW.err; exit 1; }
echo pmcW ok
