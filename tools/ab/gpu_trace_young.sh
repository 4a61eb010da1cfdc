# Kernel trace of one C4 shard (rehearsal of shard 0 of 2, 5 timed ticks) with young tiles:
# per-kernel durations and gaps per tick.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/trace_young -o run --output-format csv -- python $R/bench.py --rehearse-shards 2 --steps 5 --warmup 5 --no-cpu-baseline > $R/gpurun_out/trace_young.json 2> $R/gpurun_out/trace_young.err || { echo "trace failed"; tail -5 $R/gpurun_out/trace_young.err; exit 1; }
echo trace done
