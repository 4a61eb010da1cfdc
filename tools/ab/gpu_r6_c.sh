# Round 6: per-tick pull counters of the 8-shard rank (tools/diag_ticks.py), the new library (lib/r6a)
# and the round-5 one, concurrent kernels and (young_overlap 0) one after the other.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for v in r6a r5; do
  for ov in 1 0; do
    GOSSIP_YOUNG_OVERLAP=$ov GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/$v/libgossip.so timeout -k 10 300 python -u tools/diag_ticks.py --shards 8 --shard 1 --ticks 16 > gpurun_out/r6c_${v}_ov$ov.jsonl 2> gpurun_out/r6c_${v}_ov$ov.err || { tail -5 gpurun_out/r6c_${v}_ov$ov.err; exit 1; }
  done
done
echo done
