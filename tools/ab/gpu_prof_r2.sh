# Round-2 profile of the driver's bench command (python bench.py --steps 20 --warmup 5):
# kernel trace + stats, then one PMC pass each for FETCH_SIZE and WRITE_SIZE (pull kernels only).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2_trace -o run --output-format csv -- $B > $R/gpurun_out/r2_trace.json 2> $R/gpurun_out/r2_trace.err || { echo "trace failed"; tail -3 $R/gpurun_out/r2_trace.err; exit 1; }
echo trace ok
timeout -s KILL 400 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r2_pmcF -o run --output-format csv -- $B > $R/gpurun_out/r2_pmcF.json 2> $R/gpurun_out/r2_pmcF.err || { echo "pmcF failed"; tail -3 $R/gpurun_out/r2_pmcF.err; exit 1; }
echo pmcF ok
timeout -s KILL 400 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r2_pmcW -o run --output-format csv -- $B > $R/gpurun_out/r2_pmcW.json 2> $R/gpurun_out/r2_pmcW.err || { echo "pmcW failed"; tail -3 $R/gpurun_out/r2_pmcW.err; exit 1; }
echo pmcW ok
