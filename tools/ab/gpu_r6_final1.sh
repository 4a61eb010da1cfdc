# Round 6 final evidence, part 1: the driver's C4 command with its CPU baseline, the rocprofv3 kernel
# trace + stats of the same command, and its two PMC passes (FETCH_SIZE, WRITE_SIZE) ->
# profiles/pmc_C4*.json keyed by this build (tools/pmc_traffic.py --bench-json).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6f1_bench.json 2> gpurun_out/r6f1_bench.err || { tail -5 gpurun_out/r6f1_bench.err; exit 1; }
python tools/ab_line.py final gpurun_out/r6f1_bench.json
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6f1_trace -o run --output-format csv -- $B > $R/gpurun_out/r6f1_trace.json 2> $R/gpurun_out/r6f1_trace.err || { echo "trace failed"; tail -3 $R/gpurun_out/r6f1_trace.err; exit 1; }
echo trace ok
timeout -s KILL 450 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r6f1_pmcF -o run --output-format csv -- $B > $R/gpurun_out/r6f1_pmcF.json 2> $R/gpurun_out/r6f1_pmcF.err || { echo "pmcF failed"; tail -3 $R/gpurun_out/r6f1_pmcF.err; exit 1; }
echo pmcF ok
timeout -s KILL 450 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r6f1_pmcW -o run --output-format csv -- $B > $R/gpurun_out/r6f1_pmcW.json 2> $R/gpurun_out/r6f1_pmcW.err || { echo "pmcW failed"; tail -3 $R/gpurun_out/r6f1_pmcW.err; exit 1; }
echo pmcW ok
cd $R
python tools/prof_summary.py gpurun_out/r6f1_trace run --timed 20 --passes 2 --phase-with k_pull_young --out gpurun_out/r6f1_kernel_summary.json | tail -5
F=$(ls gpurun_out/r6f1_pmcF/*counter_collection.csv | head -1); W=$(ls gpurun_out/r6f1_pmcW/*counter_collection.csv | head -1)
python tools/pmc_traffic.py $F $W --timed 20 --passes 2 --kernel "k_pull<" --bench-json gpurun_out/r6f1_pmcF.json --out gpurun_out/pmc_C4.json | tail -4
python tools/pmc_traffic.py $F $W --timed 14 --passes 2 --kernel "k_pull_young" --bench-json gpurun_out/r6f1_pmcF.json --out gpurun_out/pmc_C4_young.json | tail -4
