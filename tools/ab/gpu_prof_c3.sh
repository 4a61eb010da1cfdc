# Round 3: the C3 line (1M nodes, avg degree 16) -- bench.py --workload C3 with and without young
# tiles (the auto rule's threshold sits at 2^20 nodes, just above C3), the kernel trace + stats of
# the default line, and one PMC pass each for FETCH_SIZE / WRITE_SIZE of the pull kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B="bench.py --gpus 1 --workload C3 --steps 20 --warmup 5 --no-cpu-baseline"
for y in 0 1; do
  GOSSIP_YOUNG=$y timeout -k 10 300 python $B > gpurun_out/r3_c3_young$y.json 2> gpurun_out/r3_c3_young$y.err || { echo "c3 young=$y failed"; tail -3 gpurun_out/r3_c3_young$y.err; exit 1; }
  python tools/ab_line.py young$y gpurun_out/r3_c3_young$y.json
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3_c3_trace -o run --output-format csv -- python $R/$B > $R/gpurun_out/r3_c3_trace.json 2> $R/gpurun_out/r3_c3_trace.err || { echo "trace failed"; tail -3 $R/gpurun_out/r3_c3_trace.err; exit 1; }
echo trace ok
timeout -s KILL 400 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r3_c3_pmcF -o run --output-format csv -- python $R/$B > $R/gpurun_out/r3_c3_pmcF.json 2> $R/gpurun_out/r3_c3_pmcF.err || { echo "pmcF failed"; tail -3 $R/gpurun_out/r3_c3_pmcF.err; exit 1; }
echo pmcF ok
timeout -s KILL 400 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r3_c3_pmcW -o run --output-format csv -- python $R/$B > $R/gpurun_out/r3_c3_pmcW.json 2> $R/gpurun_out/r3_c3_pmcW.err || { echo "pmcW failed"; tail -3 $R/gpurun_out/r3_c3_pmcW.err; exit 1; }
echo pmcW ok
