# Round 6: empty-slot skipping (young_skip) + push marks (pull_push): parity tests of the young and
# engine suites, then every rank of the 8-shard C4 layout with the round-5 library (lib/r5) and the
# new one (lib/r6a), one after another on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest tests/test_engine_gpu.py -k "push_marks or sharded or wide or tile_list" -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r6b_tests.log 2>&1 || { tail -30 gpurun_out/r6b_tests.log; exit 1; }
tail -2 gpurun_out/r6b_tests.log
summ() {
python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print(sys.argv[1], "max", round(d["ms_per_step"], 2), "rank ms/tick", [round(x, 2) for x in c["rank_ms_per_step"]],
      "phase", [round(x, 2) for x in c["rank_phase_ms_per_tick"]], "words", c["rank_live_words"], "cap", c["rank_window_capacity_words"],
      "projected %.4e" % c["projected_job_value"], flush=True)
PY
}
for v in r6a r5; do
  GOSSIP_LIB_PATH=$R/p2p-gossip-simulation-ns3_amd/lib/$v/libgossip.so timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 --rehearse-index -1 > gpurun_out/r6b_s8all_$v.json 2> gpurun_out/r6b_s8all_$v.err || { tail -5 gpurun_out/r6b_s8all_$v.err; exit 1; }
  summ gpurun_out/r6b_s8all_$v.json
done
