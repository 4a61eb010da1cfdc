# Round 5: k_pull_young after the group-mask change: the young and engine tests, then one PMC pass
# (SQ_INSTS_VALU / LDS / SALU, SQ_WAVES) per build on the C4 line -- the product build and the
# YOUNG_DUP=k builds (lib/yd_k): 4 dedup, 6 dense rows, 9 list write + touched reset, 10 kept-entry scan.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 800 python -u -m pytest tests/test_young_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5o_tests.log 2>&1 || { tail -40 gpurun_out/r5o_tests.log; exit 1; }
tail -1 gpurun_out/r5o_tests.log
cd /tmp && export TMPDIR=/tmp
L=$R/p2p-gossip-simulation-ns3_amd/lib
for v in base 4 6 9 10; do
  lib=$L/libgossip.so; [ $v != base ] && lib=$L/yd_$v/libgossip.so
  GOSSIP_LIB_PATH=$lib timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull_young" --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/r5o_$v -o run --output-format csv -- python $R/bench.py --steps 4 --warmup 4 --no-cpu-baseline > $R/gpurun_out/r5o_$v.json 2> $R/gpurun_out/r5o_$v.err || { echo "pmc $v failed"; tail -3 $R/gpurun_out/r5o_$v.err; exit 1; }
  echo "== $v"; python $R/tools/pmc_counters.py --timed 4 --kernel k_pull_young $R/gpurun_out/r5o_$v/run_counter_collection.csv
done
