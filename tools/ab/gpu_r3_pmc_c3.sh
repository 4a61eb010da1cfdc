# Round 3: PMC HBM traffic of the C3 pull under `bench.py --workload C3 --steps 40 --warmup 30`.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r3c3_pmcF -o run --output-format csv -- $B > $R/gpurun_out/r3c3_pmcF.json 2> $R/gpurun_out/r3c3_pmcF.err || { echo "pmcF failed"; tail -3 $R/gpurun_out/r3c3_pmcF.err; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r3c3_pmcW -o run --output-format csv -- $B > $R/gpurun_out/r3c3_pmcW.json 2> $R/gpurun_out/r3c3_pmcW.err || { echo "pmcW failed"; tail -3 $R/gpurun_out/r3c3_pmcW.err; exit 1; }
echo pmc ok
cd $R
timeout -k 10 200 python bench.py --workload C3 --steps 40 --warmup 30 > gpurun_out/r3c3_line.json 2> gpurun_out/r3c3_line.err || { tail -3 gpurun_out/r3c3_line.err; exit 1; }
python tools/ab_line.py c3 gpurun_out/r3c3_line.json
