# Round 5: PMC traffic passes (FETCH_SIZE, WRITE_SIZE) of one rank of 8 shards at the new default
# (tick rule, fresh tile per birth tick); tools/pmc_traffic.py afterwards on the CPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8"
timeout -k 10 300 $B > $R/gpurun_out/r5z6_s8_line.json 2> $R/gpurun_out/r5z6_s8_line.err || { echo "line failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r5z6_pmcF -o run --output-format csv -- $B > $R/gpurun_out/r5z6_pmcF.json 2> $R/gpurun_out/r5z6_pmcF.err || { echo "pmcF failed"; tail -3 $R/gpurun_out/r5z6_pmcF.err; exit 1; }
echo pmcF ok
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r5z6_pmcW -o run --output-format csv -- $B > $R/gpurun_out/r5z6_pmcW.json 2> $R/gpurun_out/r5z6_pmcW.err || { echo "pmcW failed"; tail -3 $R/gpurun_out/r5z6_pmcW.err; exit 1; }
echo pmcW ok
