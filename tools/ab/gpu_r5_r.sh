# Round 5: k_pull SP also fixes shared outputs (young alongside) and no snapshot count (static VALU
# 1648 -> 1464, readlanes 232 -> 126):
# C4 / young / engine parity, then a same-box A/B of the C4 line against the build before it
# (lib/var_p3) and one PMC pass of k_pull's SQ instruction counts per build.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest tests/test_scale_gpu.py -k "c4" -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r5r_c4_tests.log 2>&1 || { tail -40 gpurun_out/r5r_c4_tests.log; exit 1; }
tail -1 gpurun_out/r5r_c4_tests.log
timeout -k 10 800 python -u -m pytest tests/test_engine_gpu.py tests/test_late_exit_gpu.py tests/test_c3_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5r_tests.log 2>&1 || { tail -40 gpurun_out/r5r_tests.log; exit 1; }
tail -1 gpurun_out/r5r_tests.log
L=$R/p2p-gossip-simulation-ns3_amd/lib
for rep in 1 2; do
  for v in sp prev; do
    lib=$L/libgossip.so; [ $v = prev ] && lib=$L/var_p3/libgossip.so
    GOSSIP_LIB_PATH=$lib timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5r_${v}$rep.json 2> gpurun_out/r5r_${v}$rep.err || { tail -5 gpurun_out/r5r_${v}$rep.err; exit 1; }
    python tools/ab_line.py ${v}$rep gpurun_out/r5r_${v}$rep.json
  done
done
cd /tmp && export TMPDIR=/tmp
for v in sp prev; do
  lib=$L/libgossip.so; [ $v = prev ] && lib=$L/var_p3/libgossip.so
  GOSSIP_LIB_PATH=$lib timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull<" --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/r5r_pmc_$v -o run --output-format csv -- python $R/bench.py --steps 4 --warmup 4 --no-cpu-baseline > $R/gpurun_out/r5r_pmc_$v.json 2> $R/gpurun_out/r5r_pmc_$v.err || { echo "pmc $v failed"; tail -3 $R/gpurun_out/r5r_pmc_$v.err; exit 1; }
  echo "== $v"; python $R/tools/pmc_counters.py --timed 4 --kernel "k_pull<" $R/gpurun_out/r5r_pmc_$v/run_counter_collection.csv
done
