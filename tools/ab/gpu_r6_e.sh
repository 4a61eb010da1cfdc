# Round 6: push tiles keep their trusted sat bits (lib/r6c): push / engine parity tests, then the C4
# N = 1 line with push marks auto / off and the round-5 library, and every rank of 8, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py -k "push or sat or sharded or wide or tile_list" -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r6e_tests.log 2>&1 || { tail -30 gpurun_out/r6e_tests.log; exit 1; }
tail -1 gpurun_out/r6e_tests.log
L=$R/p2p-gossip-simulation-ns3_amd/lib
run() {  # name lib env...
  local name=$1 lib=$2; shift 2
  env GOSSIP_LIB_PATH=$L/$lib/libgossip.so "$@" timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r6e_$name.json 2> gpurun_out/r6e_$name.err || { tail -5 gpurun_out/r6e_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r6e_$name.json
}
run c4_r6c r6c X=1
run c4_r6c_nopush r6c GOSSIP_PULL_PUSH=0
run c4_r5 r5 X=1
run c4_r6c_2 r6c X=1
GOSSIP_LIB_PATH=$L/r6c/libgossip.so timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 --rehearse-index -1 > gpurun_out/r6e_s8all.json 2> gpurun_out/r6e_s8all.err || { tail -5 gpurun_out/r6e_s8all.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r6e_s8all.json").read().strip().splitlines()[-1])
c = d["config"]
print("s8all max", round(d["ms_per_step"], 2), [round(x, 2) for x in c["rank_ms_per_step"]], "projected %.4e" % c["projected_job_value"])
PY
