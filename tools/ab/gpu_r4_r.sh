# Round 4: k_pull_young variants on one box, then the device-stamped DENSE phase timer: A = unused peer groups not issued + slot headers by
# lead-lane ballots (71 VGPRs), B = header ballots only (67 VGPRs), against the final tree (64).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4r_$name.json 2> gpurun_out/r4r_$name.err || { tail -5 gpurun_out/r4r_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4r_$name.json
}
L=$R/p2p-gossip-simulation-ns3_amd/lib
run now
run a GOSSIP_LIB_PATH=$L/ab_a/libgossip.so
run b GOSSIP_LIB_PATH=$L/ab_b/libgossip.so
run now_seq GOSSIP_YOUNG_OVERLAP=0
run a_seq GOSSIP_LIB_PATH=$L/ab_a/libgossip.so GOSSIP_YOUNG_OVERLAP=0
run b_seq GOSSIP_LIB_PATH=$L/ab_b/libgossip.so GOSSIP_YOUNG_OVERLAP=0
run now2
# the DENSE phase timed by device stamps (first k_transpose block start -> last k_dense_dedup
# block end): dense parity, the C2 / C5 lines and the C2 trace to compare the span with
timeout -k 10 400 python -u -m pytest "tests/test_scale_gpu.py::test_c2_full_run_all_paths_match_oracle_b" "tests/test_scale_gpu.py::test_c2_golden_fixture_on_every_path" "tests/test_scale_gpu.py::test_c5_mfma_equals_csr_and_oracle_b" tests/test_hop_batch.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4r_dense_tests.log 2>&1 || { tail -30 gpurun_out/r4r_dense_tests.log; exit 1; }
tail -2 gpurun_out/r4r_dense_tests.log
timeout -k 10 300 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/r4r_c2.json 2> gpurun_out/r4r_c2.err || { tail -5 gpurun_out/r4r_c2.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r4r_c2.json').read().strip().splitlines()[-1]);print({k:v for k,v in d.items() if 'util' in k or 'ms_avg' in k})"
timeout -k 10 300 python tools/bench_dense.py c5 --modes dense > gpurun_out/r4r_c5.json 2> gpurun_out/r4r_c5.err || { tail -5 gpurun_out/r4r_c5.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4r_c2trace -o run --output-format csv -- python $R/tools/bench_dense.py c2 --batch --modes dense > $R/gpurun_out/r4r_c2trace.json 2> $R/gpurun_out/r4r_c2trace.err || { echo "c2 trace failed"; tail -3 $R/gpurun_out/r4r_c2trace.err; exit 1; }
echo c2 trace ok
