# Round 5: rocprofv3 kernel trace of one rank of 8 shards (per-dispatch durations by tick age).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5u_s8_trace -o run --output-format csv -- $B > $R/gpurun_out/r5u_s8_trace.json 2> $R/gpurun_out/r5u_s8_trace.err || { echo "trace failed"; tail -3 $R/gpurun_out/r5u_s8_trace.err; exit 1; }
echo trace ok
