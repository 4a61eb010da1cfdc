# PMC passes for the default C4 bench (separate runs, counters only): FETCH_SIZE, WRITE_SIZE.
# Then: python tools/pmc_traffic.py ... --timed 40 --passes 2 --out profiles/pmc_C4.json
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pmcF_c4 -o run --output-format csv -- python $R/bench.py --no-cpu-baseline > $R/gpurun_out/pmcF_c4.json 2> $R/gpurun_out/pmcF_c4.err || { echo "pmcF failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/pmcW_c4 -o run --output-format csv -- python $R/bench.py --no-cpu-baseline > $R/gpurun_out/pmcW_c4.json 2> $R/gpurun_out/pmcW_c4.err || { echo "pmcW failed"; exit 1; }
echo pmc done
