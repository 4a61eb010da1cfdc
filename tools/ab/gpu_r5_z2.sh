# Round 5 final evidence, part 2: the driver's C4 command with its CPU baseline, the rocprofv3
# kernel trace + stats of the same command, and its two PMC passes (FETCH_SIZE, WRITE_SIZE) ->
# profiles/pmc_C4*.json keyed by this build (tools/pmc_traffic.py --bench-json); then the C3 line,
# trace and PMC passes (profiles/pmc_C3.json).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5z2_bench.json 2> gpurun_out/r5z2_bench.err || { tail -5 gpurun_out/r5z2_bench.err; exit 1; }
python tools/ab_line.py final gpurun_out/r5z2_bench.json
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5z2_trace -o run --output-format csv -- $B > $R/gpurun_out/r5z2_trace.json 2> $R/gpurun_out/r5z2_trace.err || { echo "trace failed"; tail -3 $R/gpurun_out/r5z2_trace.err; exit 1; }
echo trace ok
timeout -s KILL 450 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r5z2_pmcF -o run --output-format csv -- $B > $R/gpurun_out/r5z2_pmcF.json 2> $R/gpurun_out/r5z2_pmcF.err || { echo "pmcF failed"; tail -3 $R/gpurun_out/r5z2_pmcF.err; exit 1; }
echo pmcF ok
timeout -s KILL 450 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r5z2_pmcW -o run --output-format csv -- $B > $R/gpurun_out/r5z2_pmcW.json 2> $R/gpurun_out/r5z2_pmcW.err || { echo "pmcW failed"; tail -3 $R/gpurun_out/r5z2_pmcW.err; exit 1; }
echo pmcW ok
cd $R
C3="python bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline"
timeout -k 10 300 $C3 > gpurun_out/r5z2_c3.json 2> gpurun_out/r5z2_c3.err || { tail -5 gpurun_out/r5z2_c3.err; exit 1; }
python tools/ab_line.py c3 gpurun_out/r5z2_c3.json
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5z2_c3trace -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r5z2_c3trace.json 2> $R/gpurun_out/r5z2_c3trace.err || { echo "c3 trace failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r5z2_c3pmcF -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r5z2_c3pmcF.json 2> $R/gpurun_out/r5z2_c3pmcF.err || { echo "c3 pmcF failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r5z2_c3pmcW -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r5z2_c3pmcW.json 2> $R/gpurun_out/r5z2_c3pmcW.err || { echo "c3 pmcW failed"; exit 1; }
echo c3 done
