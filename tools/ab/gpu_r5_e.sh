# Round 5: the fused DENSE kernel with data-parallel rounds + a stream-K tail -- parity first, then
# the C2 / C5 lines, their traces, and the DENSE_STAMPS diagnostic build (lib/diag_ds) on both.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_dense_fused_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/r5e_fused_tests.log 2>&1 || { tail -40 gpurun_out/r5e_fused_tests.log; exit 1; }
tail -1 gpurun_out/r5e_fused_tests.log
timeout -k 10 900 python -u -m pytest tests/test_hop_batch.py tests/test_scale_gpu.py -k "c2 or c5 or hop_batch" -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r5e_dense_tests.log 2>&1 || { tail -40 gpurun_out/r5e_dense_tests.log; exit 1; }
tail -1 gpurun_out/r5e_dense_tests.log
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "dense_mfma" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5e_dense2_tests.log 2>&1 || { tail -40 gpurun_out/r5e_dense2_tests.log; exit 1; }
tail -1 gpurun_out/r5e_dense2_tests.log
for c in "c2 --batch" "c5"; do
  n=$(echo $c | cut -d' ' -f1)
  timeout -k 10 400 python tools/bench_dense.py $c --modes dense > gpurun_out/r5e_$n.json 2> gpurun_out/r5e_$n.err || { tail -5 gpurun_out/r5e_$n.err; exit 1; }
  cat gpurun_out/r5e_$n.json
  GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/diag_ds/libgossip.so timeout -k 10 400 python tools/bench_dense.py $c --modes dense > gpurun_out/r5e_${n}_ds.json 2> gpurun_out/r5e_${n}_ds.err || { tail -5 gpurun_out/r5e_${n}_ds.err; exit 1; }
  grep dense_stamps gpurun_out/r5e_${n}_ds.err | tail -1
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5e_c2trace -o run --output-format csv -- python $R/tools/bench_dense.py c2 --batch --modes dense > $R/gpurun_out/r5e_c2trace.json 2> $R/gpurun_out/r5e_c2trace.err || { echo "c2 trace failed"; tail -3 $R/gpurun_out/r5e_c2trace.err; exit 1; }
echo c2 trace ok
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5e_c5trace -o run --output-format csv -- python $R/tools/bench_dense.py c5 --modes dense > $R/gpurun_out/r5e_c5trace.json 2> $R/gpurun_out/r5e_c5trace.err || { echo "c5 trace failed"; tail -3 $R/gpurun_out/r5e_c5trace.err; exit 1; }
echo c5 trace ok
