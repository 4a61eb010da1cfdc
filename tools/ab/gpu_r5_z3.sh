# Round 5: the birth-tick rule with a fresh tile per birth tick (bench.shard_flags): sharded
# engines sum to the whole engine under every rule, then one rank of 8 shards at the new default
# and the 8-shard rank's kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k "sharded or shard" -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5z3_tests.log 2>&1 || { tail -40 gpurun_out/r5z3_tests.log; exit 1; }
tail -1 gpurun_out/r5z3_tests.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 > gpurun_out/r5z3_s8.json 2> gpurun_out/r5z3_s8.err || { tail -5 gpurun_out/r5z3_s8.err; exit 1; }
python tools/ab_line.py s8 gpurun_out/r5z3_s8.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5z3_s8_trace -o run --output-format csv -- python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 > $R/gpurun_out/r5z3_s8_trace.json 2> $R/gpurun_out/r5z3_s8_trace.err || { echo "trace failed"; exit 1; }
echo trace ok
