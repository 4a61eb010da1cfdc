# Round 3 diagnostic: how many of k_pull's own-seen pair reads are in tiles that want no bit
# (saturated node-tiles)?  The PULL_DIAG_SAT build reports that count in the occupancy slot.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/ab/diag.so timeout -k 10 200 python bench.py --rehearse-shards 2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3sat.json 2> gpurun_out/r3sat.err || { tail -5 gpurun_out/r3sat.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r3sat.json').read().strip().splitlines()[-1]);b=d['roofline']['kernels']['k_pull']['bytes_breakdown_per_launch']
print('seen pairs read: %.2f GB; of them in tiles wanting no bit: %.2f GB (x2: the 8-B count is 16-B pairs)'%(b['own_seen_read']/1e9, 2*b['peer_occupancy']/1e9))"
