# Round 6: the birth-tick rule with a 4-tick cycle (engine option shard_period; each birth-tick class
# split over 2 shards by hash) against the 8-tick rule -- every rank of the 8-GPU C4 layout rehearsed
# at the driver's arguments, one box; the per-tick table of rank 1; the sharded-sum parity test.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 200 python -u -m pytest tests/test_engine_gpu.py -k sharded_engines -x -q --timeout 120 --timeout-method thread > gpurun_out/r6n_tests.log 2>&1 || { tail -20 gpurun_out/r6n_tests.log; exit 1; }
tail -1 gpurun_out/r6n_tests.log
for P in 4 8; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 --rehearse-index -1 --shard-period $P > gpurun_out/r6n_s8all_p$P.json 2> gpurun_out/r6n_s8all_p$P.err || { tail -5 gpurun_out/r6n_s8all_p$P.err; exit 1; }
  python - $P <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/r6n_s8all_p{sys.argv[1]}.json").read().strip().splitlines()[-1]); c = d["config"]
r = c["rank_ms_per_step"]
print("P", sys.argv[1], "max %.2f mean %.2f" % (max(r), sum(r) / len(r)), [round(x, 2) for x in r], "projected %.4e" % c["projected_job_value"], "period", c.get("shard_period"))
PY
done
timeout -k 10 300 python -u tools/diag_ticks.py --shards 8 --shard 1 --ticks 16 --option shard_period=4 > gpurun_out/r6n_diag_p4.jsonl 2> gpurun_out/r6n_diag_p4.err || { tail -5 gpurun_out/r6n_diag_p4.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r6n_diag_p4.jsonl"):
    d = json.loads(l)
    print(d["tick"], "phase %.2f pull %.2f young %.2f" % (d["pull_phase_ms"], d["pull_ms"], d["young_ms"]))
PY
