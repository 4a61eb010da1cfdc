# Round 6: k_pull_young's per-segment shader cycles (YOUNG_STAMPS build, lib/ys) on every tick of
# rank 1 of the 8-shard C4 layout (tools/diag_ticks.py): where the ages-3/4 ticks' walk goes.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ys/libgossip.so timeout -k 10 300 python -u tools/diag_ticks.py --shards 8 --shard 1 --ticks 16 > gpurun_out/r6m_diag_ys.jsonl 2> gpurun_out/r6m_diag_ys.err || { tail -5 gpurun_out/r6m_diag_ys.err; exit 1; }
grep -c young_stamps gpurun_out/r6m_diag_ys.err
