# Round 3: k_pull whole seen lines (pull_seen_lines 0 / 1): C4 shard time A/B, then PMC
# FETCH_SIZE / WRITE_SIZE of k_pull<32,1,true> for both (5 timed ticks each).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "tile_list or work_skipping or wide_window" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3l_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r3l_tests.log; [ $rc -eq 0 ] || exit 1
GOSSIP_PULL_SEEN_LINES=1 timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_late_exit_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3l_tests1.log 2>&1
rc=$?; tail -2 gpurun_out/r3l_tests1.log; [ $rc -eq 0 ] || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3l_$name.json 2> gpurun_out/r3l_$name.err || { tail -5 gpurun_out/r3l_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r3l_$name.json
}
run sl0 GOSSIP_PULL_SEEN_LINES=0
run sl1 GOSSIP_PULL_SEEN_LINES=1
cd /tmp && export TMPDIR=/tmp
for sl in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    GOSSIP_PULL_SEEN_LINES=$sl timeout -s KILL 200 rocprofv3 --kernel-include-regex "k_pull<32" --pmc $c -d $R/gpurun_out/r3l_pmc_${sl}_$c -o run --output-format csv -- python $R/bench.py --rehearse-shards 2 --steps 5 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r3l_pmc_${sl}_$c.json 2> $R/gpurun_out/r3l_pmc_${sl}_$c.err || { echo "pmc $sl $c failed"; tail -3 $R/gpurun_out/r3l_pmc_${sl}_$c.err; exit 1; }
    echo "sl=$sl $c"; python $R/tools/pmc_counters.py --timed 5 --kernel "k_pull<32" $R/gpurun_out/r3l_pmc_${sl}_$c/run_counter_collection.csv
  done
done
