# Round 5, baseline of the round-4 dense path on this round's boxes: C2 hop-batched and C5 at its
# BASELINE width (4,096 shares), lines + rocprofv3 kernel traces (per-dispatch durations).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/r5a_c2.json 2> gpurun_out/r5a_c2.err || { tail -5 gpurun_out/r5a_c2.err; exit 1; }
cat gpurun_out/r5a_c2.json
timeout -k 10 400 python tools/bench_dense.py c5 --modes dense > gpurun_out/r5a_c5.json 2> gpurun_out/r5a_c5.err || { tail -5 gpurun_out/r5a_c5.err; exit 1; }
cat gpurun_out/r5a_c5.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5a_c2trace -o run --output-format csv -- python $R/tools/bench_dense.py c2 --batch --modes dense > $R/gpurun_out/r5a_c2trace.json 2> $R/gpurun_out/r5a_c2trace.err || { echo "c2 trace failed"; tail -3 $R/gpurun_out/r5a_c2trace.err; exit 1; }
echo c2 trace ok
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5a_c5trace -o run --output-format csv -- python $R/tools/bench_dense.py c5 --modes dense > $R/gpurun_out/r5a_c5trace.json 2> $R/gpurun_out/r5a_c5trace.err || { echo "c5 trace failed"; tail -3 $R/gpurun_out/r5a_c5trace.err; exit 1; }
echo c5 trace ok
