# Round 6 baseline: every rank of the 8-shard C4 layout (bench default: birth-tick rule, fresh tile
# per birth tick), rehearsed one after another on one GPU, with the round-5 library (lib/r5).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/r5/libgossip.so timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 --rehearse-index -1 > gpurun_out/r6a_s8all.json 2> gpurun_out/r6a_s8all.err || { tail -5 gpurun_out/r6a_s8all.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r6a_s8all.json").read().strip().splitlines()[-1])
c = d["config"]
print("rank ms/tick", [round(x, 2) for x in c["rank_ms_per_step"]])
print("rank phase", [round(x, 2) for x in c["rank_phase_ms_per_tick"]])
print("words", c["rank_live_words"], "cap", c["rank_window_capacity_words"])
print("projected", c["projected_job_value"])
PY
