# Round 6: k_dense_fused with the two waves of each SIMD taking turns at issue priority (s_setprio,
# half a stage each; DENSE_PRIO build, lib/prio) against the product build, same box: C2 / C5 lines
# twice each, then the DENSE_STAMPS breakdown of both (lib/prio_ds, lib/ds).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
L=$R/p2p-gossip-simulation-ns3_amd/lib
for rep in 1 2; do
  for v in base prio; do
    lp=$L/libgossip.so; [ $v = prio ] && lp=$L/prio/libgossip.so
    for c in c2 c5; do
      a="$c"; [ $c = c2 ] && a="c2 --batch"
      GOSSIP_LIB_PATH=$lp timeout -k 10 300 python tools/bench_dense.py $a --modes dense > gpurun_out/r6o_${v}_${c}_$rep.json 2> gpurun_out/r6o_${v}_${c}_$rep.err || { tail -5 gpurun_out/r6o_${v}_${c}_$rep.err; exit 1; }
      echo -n "$v rep$rep "; python tools/ab_dense.py $c gpurun_out/r6o_${v}_${c}_$rep.json
    done
  done
done
for v in ds prio_ds; do
  for c in c2 c5; do
    a="$c"; [ $c = c2 ] && a="c2 --batch"
    GOSSIP_LIB_PATH=$L/$v/libgossip.so timeout -k 10 300 python tools/bench_dense.py $a --modes dense > gpurun_out/r6o_${v}_$c.json 2> gpurun_out/r6o_${v}_$c.err || { tail -5 gpurun_out/r6o_${v}_$c.err; exit 1; }
    echo -n "$v $c "; grep dense_stamps gpurun_out/r6o_${v}_$c.err | tail -1
  done
done
