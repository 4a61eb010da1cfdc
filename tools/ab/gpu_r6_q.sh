# Round 6: k_dense_fused issuing the next stage's LDS-DMA pieces after the unit's first (li1) or second
# (li2) 128-k slice of MFMAs instead of right after the stage barrier (DENSE_LATE_ISSUE builds,
# lib/li1, lib/li2) against the product build, same box: fused parity tests on li1, the C2 / C5 lines
# twice each, then the DENSE_STAMPS breakdown of li1 and of the product build (lib/li1ds, lib/ds).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
L=$R/p2p-gossip-simulation-ns3_amd/lib
GOSSIP_LIB_PATH=$L/li1/libgossip.so timeout -k 10 400 python -u -m pytest tests/test_dense_fused_gpu.py tests/test_row_partition.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/r6q_tests.log 2>&1 || { tail -30 gpurun_out/r6q_tests.log; exit 1; }
tail -1 gpurun_out/r6q_tests.log
for rep in 1 2; do
  for v in base li1 li2; do
    lp=$L/libgossip.so; [ $v != base ] && lp=$L/$v/libgossip.so
    for c in c2 c5; do
      a="$c"; [ $c = c2 ] && a="c2 --batch"
      GOSSIP_LIB_PATH=$lp timeout -k 10 300 python tools/bench_dense.py $a --modes dense > gpurun_out/r6q_${v}_${c}_$rep.json 2> gpurun_out/r6q_${v}_${c}_$rep.err || { tail -5 gpurun_out/r6q_${v}_${c}_$rep.err; exit 1; }
      echo -n "$v rep$rep "; python tools/ab_dense.py $c gpurun_out/r6q_${v}_${c}_$rep.json
    done
  done
done
for v in ds li1ds; do
  for c in c2 c5; do
    a="$c"; [ $c = c2 ] && a="c2 --batch"
    GOSSIP_LIB_PATH=$L/$v/libgossip.so timeout -k 10 300 python tools/bench_dense.py $a --modes dense > gpurun_out/r6q_${v}_$c.json 2> gpurun_out/r6q_${v}_$c.err || { tail -5 gpurun_out/r6q_${v}_$c.err; exit 1; }
    echo -n "$v $c "; grep dense_stamps gpurun_out/r6q_${v}_$c.err | tail -1
  done
done
