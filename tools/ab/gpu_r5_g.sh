# Round 5: k_dense_fused with merged prologue loads, deferred whole-tile epilogues and no-return
# liveness atomics: parity, then a same-box A/B of the C2 / C5 lines against the previous build
# (lib/var_r5f), the DENSE_STAMPS build and the C2 / C5 traces of this tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_dense_fused_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/r5g_fused_tests.log 2>&1 || { tail -40 gpurun_out/r5g_fused_tests.log; exit 1; }
tail -1 gpurun_out/r5g_fused_tests.log
timeout -k 10 900 python -u -m pytest tests/test_hop_batch.py tests/test_scale_gpu.py -k "c2 or c5 or hop_batch" -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r5g_dense_tests.log 2>&1 || { tail -40 gpurun_out/r5g_dense_tests.log; exit 1; }
tail -1 gpurun_out/r5g_dense_tests.log
L=$R/p2p-gossip-simulation-ns3_amd/lib
for rep in 1 2; do
for c in "c2 --batch" "c5"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -k 10 400 python tools/bench_dense.py $c --modes dense > gpurun_out/r5g_${n}_cur$rep.json 2> gpurun_out/r5g_${n}_cur$rep.err || { tail -5 gpurun_out/r5g_${n}_cur$rep.err; exit 1; }
  python tools/ab_dense.py cur$rep gpurun_out/r5g_${n}_cur$rep.json
  GOSSIP_LIB_PATH=$L/var_r5f/libgossip.so timeout -k 10 400 python tools/bench_dense.py $c --modes dense > gpurun_out/r5g_${n}_prev$rep.json 2> gpurun_out/r5g_${n}_prev$rep.err || { tail -5 gpurun_out/r5g_${n}_prev$rep.err; exit 1; }
  python tools/ab_dense.py prev$rep gpurun_out/r5g_${n}_prev$rep.json
done
done
for c in "c2 --batch" "c5"; do
  n=$(echo $c | cut -d' ' -f1)
  GOSSIP_LIB_PATH=$L/diag_ds/libgossip.so timeout -k 10 400 python tools/bench_dense.py $c --modes dense > gpurun_out/r5g_${n}_ds.json 2> gpurun_out/r5g_${n}_ds.err || { tail -5 gpurun_out/r5g_${n}_ds.err; exit 1; }
  grep dense_stamps gpurun_out/r5g_${n}_ds.err | tail -1
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5g_c2trace -o run --output-format csv -- python $R/tools/bench_dense.py c2 --batch --modes dense > $R/gpurun_out/r5g_c2trace.json 2> $R/gpurun_out/r5g_c2trace.err || { echo "c2 trace failed"; tail -3 $R/gpurun_out/r5g_c2trace.err; exit 1; }
python $R/tools/dense_trace.py $R/gpurun_out/r5g_c2trace/run_kernel_trace.csv $R/gpurun_out/r5g_c2trace.json | grep mfma_util
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5g_c5trace -o run --output-format csv -- python $R/tools/bench_dense.py c5 --modes dense > $R/gpurun_out/r5g_c5trace.json 2> $R/gpurun_out/r5g_c5trace.err || { echo "c5 trace failed"; tail -3 $R/gpurun_out/r5g_c5trace.err; exit 1; }
python $R/tools/dense_trace.py $R/gpurun_out/r5g_c5trace/run_kernel_trace.csv $R/gpurun_out/r5g_c5trace.json | grep mfma_util
