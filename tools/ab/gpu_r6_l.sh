# Round 6: ballots four rows per wait (dense_kernel.h write_lanes4) -- fused parity tests, the C2 / C5
# lines, then the DENSE_STAMPS breakdown of the same build.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_dense_fused_gpu.py tests/test_row_partition.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r6l_tests.log 2>&1 || { tail -30 gpurun_out/r6l_tests.log; exit 1; }
tail -1 gpurun_out/r6l_tests.log
for c in c2 c5; do
  a="$c"; [ $c = c2 ] && a="c2 --batch"
  timeout -k 10 400 python tools/bench_dense.py $a --modes dense > gpurun_out/r6l_$c.json 2> gpurun_out/r6l_$c.err || { tail -5 gpurun_out/r6l_$c.err; exit 1; }
  python tools/ab_dense.py $c gpurun_out/r6l_$c.json
done
for c in c2 c5; do
  a="$c"; [ $c = c2 ] && a="c2 --batch"
  GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ds/libgossip.so timeout -k 10 300 python tools/bench_dense.py $a --modes dense > gpurun_out/r6l_ds_$c.json 2> gpurun_out/r6l_ds_$c.err || { tail -5 gpurun_out/r6l_ds_$c.err; exit 1; }
  grep dense_stamps gpurun_out/r6l_ds_$c.err | tail -1
done
