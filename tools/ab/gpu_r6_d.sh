# Round 6: + idle-node pass (k_young_idle), k_pull's idle-node skip and births' push marks (lib/r6b):
# young / engine parity tests, per-tick counters of the 8-shard rank, every rank of 8, and the C4
# N = 1 line against the round-5 library (lib/r5), same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_young_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r6d_tests.log 2>&1 || { tail -30 gpurun_out/r6d_tests.log; exit 1; }
tail -1 gpurun_out/r6d_tests.log
GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/r6b/libgossip.so timeout -k 10 300 python -u tools/diag_ticks.py --shards 8 --shard 1 --ticks 16 > gpurun_out/r6d_diag_r6b.jsonl 2> gpurun_out/r6d_diag_r6b.err || { tail -5 gpurun_out/r6d_diag_r6b.err; exit 1; }
summ() {
python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print(sys.argv[1], "max", round(d["ms_per_step"], 2), "rank ms/tick", [round(x, 2) for x in c["rank_ms_per_step"]],
      "phase", [round(x, 2) for x in c["rank_phase_ms_per_tick"]], "words", c["rank_live_words"],
      "projected %.4e" % c["projected_job_value"], flush=True)
PY
}
GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/r6b/libgossip.so timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 --rehearse-index -1 > gpurun_out/r6d_s8all_r6b.json 2> gpurun_out/r6d_s8all_r6b.err || { tail -5 gpurun_out/r6d_s8all_r6b.err; exit 1; }
summ gpurun_out/r6d_s8all_r6b.json
for v in r6b r5; do
  GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/$v/libgossip.so timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6d_c4_$v.json 2> gpurun_out/r6d_c4_$v.err || { tail -5 gpurun_out/r6d_c4_$v.err; exit 1; }
  python tools/ab_line.py c4_$v gpurun_out/r6d_c4_$v.json
done
