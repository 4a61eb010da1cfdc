# Round 4 evidence, part 1 (final tree): the driver's bench command with its CPU baselines, the
# bench with its default arguments (window headroom), the rocprofv3 kernel trace + stats of the
# driver's command, and the two PMC passes (FETCH_SIZE, WRITE_SIZE) of the same command.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4z_bench.json 2> gpurun_out/r4z_bench.err || { tail -5 gpurun_out/r4z_bench.err; exit 1; }
python tools/ab_line.py final gpurun_out/r4z_bench.json
timeout -k 10 400 python bench.py > gpurun_out/r4z_default.json 2> gpurun_out/r4z_default.err || { tail -5 gpurun_out/r4z_default.err; exit 1; }
python tools/ab_line.py default gpurun_out/r4z_default.json
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4z_trace -o run --output-format csv -- $B > $R/gpurun_out/r4z_trace.json 2> $R/gpurun_out/r4z_trace.err || { echo "trace failed"; tail -3 $R/gpurun_out/r4z_trace.err; exit 1; }
echo trace ok
timeout -s KILL 450 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r4z_pmcF -o run --output-format csv -- $B > $R/gpurun_out/r4z_pmcF.json 2> $R/gpurun_out/r4z_pmcF.err || { echo "pmcF failed"; tail -3 $R/gpurun_out/r4z_pmcF.err; exit 1; }
echo pmcF ok
timeout -s KILL 450 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r4z_pmcW -o run --output-format csv -- $B > $R/gpurun_out/r4z_pmcW.json 2> $R/gpurun_out/r4z_pmcW.err || { echo "pmcW failed"; tail -3 $R/gpurun_out/r4z_pmcW.err; exit 1; }
echo pmcW ok
