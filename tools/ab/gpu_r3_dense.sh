# Round 3: the dense (int8 MFMA) path on the round-3 build: C2 hop-batched and C5 slice lines with
# the phase timer = transpose + MFMA + dedup kernels, plus the rocprofv3 trace of C2.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/r3e_c2.json 2> gpurun_out/r3e_c2.err || { tail -5 gpurun_out/r3e_c2.err; exit 1; }
cat gpurun_out/r3e_c2.json
timeout -k 10 300 python tools/bench_dense.py c5 --modes dense > gpurun_out/r3e_c5.json 2> gpurun_out/r3e_c5.err || { tail -5 gpurun_out/r3e_c5.err; exit 1; }
cat gpurun_out/r3e_c5.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3e_trace -o run --output-format csv -- python $R/tools/bench_dense.py c2 --batch --modes dense > $R/gpurun_out/r3e_trace.json 2> $R/gpurun_out/r3e_trace.err || { echo "trace failed"; tail -3 $R/gpurun_out/r3e_trace.err; exit 1; }
echo trace ok
