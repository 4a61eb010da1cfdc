# Round 5: k_dense_fused with the epilogue's seen pairs by LDS-DMA (no register or vmcnt(0) wait
# at a tile's last stage), flags from the prologue's LDS copy, the current tile's stage mask in a
# register: parity, then a same-box A/B of the C2 / C5 lines against the previous commit's build
# (lib/var_p), the DENSE_STAMPS build and the C2 / C5 traces.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_dense_fused_gpu.py -x -v -m gpu --timeout 150 --timeout-method thread > gpurun_out/r5m_fused_tests.log 2>&1 || { tail -40 gpurun_out/r5m_fused_tests.log; exit 1; }
tail -1 gpurun_out/r5m_fused_tests.log
timeout -k 10 900 python -u -m pytest tests/test_hop_batch.py tests/test_scale_gpu.py -k "c2 or c5 or hop_batch" -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r5m_dense_tests.log 2>&1 || { tail -40 gpurun_out/r5m_dense_tests.log; exit 1; }
tail -1 gpurun_out/r5m_dense_tests.log
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -k "dense" -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5m_dense2_tests.log 2>&1 || { tail -40 gpurun_out/r5m_dense2_tests.log; exit 1; }
tail -1 gpurun_out/r5m_dense2_tests.log
L=$R/p2p-gossip-simulation-ns3_amd/lib
one() {  # name, env..., then the bench_dense args after --
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 400 python tools/bench_dense.py "$@" --modes dense > gpurun_out/r5m_$name.json 2> gpurun_out/r5m_$name.err || { tail -5 gpurun_out/r5m_$name.err; exit 1; }
  python tools/ab_dense.py $name gpurun_out/r5m_$name.json
}
for rep in 1 2; do
  for c in c2 c5; do
    a="$c"; [ $c = c2 ] && a="c2 --batch"
    one ${c}_cur$rep X=1 -- $a
    one ${c}_prev$rep GOSSIP_LIB_PATH=$L/var_p/libgossip.so -- $a
  done
done
one c2_ds GOSSIP_LIB_PATH=$L/diag_ds/libgossip.so -- c2 --batch
grep dense_stamps gpurun_out/r5m_c2_ds.err | tail -1
one c5_ds GOSSIP_LIB_PATH=$L/diag_ds/libgossip.so -- c5
grep dense_stamps gpurun_out/r5m_c5_ds.err | tail -1
cd /tmp && export TMPDIR=/tmp
for c in c2 c5; do
  a="$c"; [ $c = c2 ] && a="c2 --batch"
  timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5m_${c}trace -o run --output-format csv -- python $R/tools/bench_dense.py $a --modes dense > $R/gpurun_out/r5m_${c}trace.json 2> $R/gpurun_out/r5m_${c}trace.err || { echo "$c trace failed"; tail -3 $R/gpurun_out/r5m_${c}trace.err; exit 1; }
  python $R/tools/dense_trace.py $R/gpurun_out/r5m_${c}trace/run_kernel_trace.csv $R/gpurun_out/r5m_${c}trace.json | grep mfma_util
done
