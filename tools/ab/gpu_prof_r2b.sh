# Round-2 final profile of the driver's bench command (python bench.py --steps 20 --warmup 5)
# with k_pull and k_pull_young concurrent: kernel trace + stats, then one PMC pass each for
# FETCH_SIZE and WRITE_SIZE (both pull kernels; the profiler serialises kernels under PMC).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r2b_trace -o run --output-format csv -- $B > $R/gpurun_out/r2b_trace.json 2> $R/gpurun_out/r2b_trace.err || { echo "trace failed"; tail -3 $R/gpurun_out/r2b_trace.err; exit 1; }
echo trace ok
timeout -s KILL 400 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r2b_pmcF -o run --output-format csv -- $B > $R/gpurun_out/r2b_pmcF.json 2> $R/gpurun_out/r2b_pmcF.err || { echo "pmcF failed"; tail -3 $R/gpurun_out/r2b_pmcF.err; exit 1; }
echo pmcF ok
timeout -s KILL 400 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r2b_pmcW -o run --output-format csv -- $B > $R/gpurun_out/r2b_pmcW.json 2> $R/gpurun_out/r2b_pmcW.err || { echo "pmcW failed"; tail -3 $R/gpurun_out/r2b_pmcW.err; exit 1; }
echo pmcW ok
