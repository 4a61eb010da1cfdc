# Round 4: k_pull_young: deg and rev prefetched, single dedup pass (slot + list staging), lovf instantiation.
# young/engine parity, same-box seq A/B vs r03, the phase-stamp build (cycles per phase of the
# node loop), one SQ pass on the young kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_young_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r4h_tests.log 2>&1 || { tail -30 gpurun_out/r4h_tests.log; exit 1; }
tail -3 gpurun_out/r4h_tests.log
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4h_$name.json 2> gpurun_out/r4h_$name.err || { tail -5 gpurun_out/r4h_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4h_$name.json
}
run r03_seq GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_r03/libgossip.so GOSSIP_YOUNG_OVERLAP=0
run now_seq GOSSIP_YOUNG_OVERLAP=0
run now
run ys_seq GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab_ys/libgossip.so GOSSIP_YOUNG_OVERLAP=0
grep young_stamps gpurun_out/r4h_ys_seq.err | tail -2
cd /tmp && export TMPDIR=/tmp
B2="python $R/bench.py --rehearse-shards 2 --steps 5 --warmup 5 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/r4h_sq -o run --output-format csv -- $B2 > $R/gpurun_out/r4h_sq.json 2> $R/gpurun_out/r4h_sq.err || { echo "sq failed"; tail -3 $R/gpurun_out/r4h_sq.err; exit 1; }
for k in "k_pull<32" "k_pull_young"; do echo "$k"; python $R/tools/pmc_counters.py --timed 5 --kernel "$k" $R/gpurun_out/r4h_sq/run_counter_collection.csv; done
