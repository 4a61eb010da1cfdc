# Round 6: k_dense_fused's per-phase shader cycles (DENSE_STAMPS build, lib/ds/libgossip.so) on C2
# hop-batched and C5 -- where the non-MFMA time of C2's phase goes.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for c in c2 c5; do
  a="$c"; [ $c = c2 ] && a="c2 --batch"
  GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ds/libgossip.so timeout -k 10 300 python tools/bench_dense.py $a --modes dense > gpurun_out/r6k_$c.json 2> gpurun_out/r6k_$c.err || { tail -5 gpurun_out/r6k_$c.err; exit 1; }
  grep dense_stamps gpurun_out/r6k_$c.err | tail -2
done
