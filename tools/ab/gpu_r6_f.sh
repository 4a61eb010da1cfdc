# Round 6: push-write tiles only before a predicted light tick (lib/r6d): push / engine parity tests,
# the C4 N = 1 line against the round-5 library, and every rank of 8 at 20 and 40 timed ticks.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k "push or sharded" tests/test_dense_fused_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r6f_tests.log 2>&1 || { tail -30 gpurun_out/r6f_tests.log; exit 1; }
tail -1 gpurun_out/r6f_tests.log
L=$R/p2p-gossip-simulation-ns3_amd/lib
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  GOSSIP_LIB_PATH=$L/$lib/libgossip.so timeout -k 10 500 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/r6f_$name.json 2> gpurun_out/r6f_$name.err || { tail -5 gpurun_out/r6f_$name.err; exit 1; }
}
s8() {
python - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d["config"]
print(sys.argv[1], "max", round(d["ms_per_step"], 2), [round(x, 2) for x in c["rank_ms_per_step"]], "mean %.2f" % (sum(c["rank_ms_per_step"]) / len(c["rank_ms_per_step"])), "projected %.4e" % c["projected_job_value"], flush=True)
PY
}
run c4_r6d r6d --steps 20 --warmup 5 && python tools/ab_line.py c4_r6d gpurun_out/r6f_c4_r6d.json
run c4_r5 r5 --steps 20 --warmup 5 && python tools/ab_line.py c4_r5 gpurun_out/r6f_c4_r5.json
run s8all20 r6d --steps 20 --warmup 5 --rehearse-shards 8 --rehearse-index -1 && s8 gpurun_out/r6f_s8all20.json
run s8all40 r6d --steps 40 --warmup 30 --rehearse-shards 8 --rehearse-index -1 && s8 gpurun_out/r6f_s8all40.json
