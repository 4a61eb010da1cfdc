# Round 5: group_fix / group_expand visit only the id groups holding an incoming bit: the engine
# and young tests (id groups on every path) and C4 parity, the C4 line against the round-4
# kernels (lib/var_tl) on one box, k_pull_young's instruction counts, the C2 DENSE_STAMPS
# calibration (block time by s_memrealtime), then the shard-rule rehearsals (gpu_r5_c.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 800 python -u -m pytest tests/test_young_gpu.py tests/test_engine_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5l_tests.log 2>&1 || { tail -40 gpurun_out/r5l_tests.log; exit 1; }
tail -1 gpurun_out/r5l_tests.log
timeout -k 10 700 python -u -m pytest tests/test_scale_gpu.py -k "c4" -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r5l_c4_tests.log 2>&1 || { tail -40 gpurun_out/r5l_c4_tests.log; exit 1; }
tail -1 gpurun_out/r5l_c4_tests.log
L=$R/p2p-gossip-simulation-ns3_amd/lib
for rep in 1 2; do
  for v in cur r4; do
    lib=$L/libgossip.so; [ $v = r4 ] && lib=$L/var_tl/libgossip.so
    GOSSIP_LIB_PATH=$lib timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5l_${v}$rep.json 2> gpurun_out/r5l_${v}$rep.err || { tail -5 gpurun_out/r5l_${v}$rep.err; exit 1; }
    python tools/ab_line.py ${v}$rep gpurun_out/r5l_${v}$rep.json
  done
done
GOSSIP_LIB_PATH=$L/diag_ds/libgossip.so timeout -k 10 400 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/r5l_c2_ds.json 2> gpurun_out/r5l_c2_ds.err || { tail -5 gpurun_out/r5l_c2_ds.err; exit 1; }
python tools/ab_dense.py c2_ds gpurun_out/r5l_c2_ds.json
grep dense_stamps gpurun_out/r5l_c2_ds.err | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull_young" --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/r5l_pmc -o run --output-format csv -- python $R/bench.py --steps 4 --warmup 4 --no-cpu-baseline > $R/gpurun_out/r5l_pmc.json 2> $R/gpurun_out/r5l_pmc.err || { echo "pmc failed"; tail -3 $R/gpurun_out/r5l_pmc.err; exit 1; }
python $R/tools/pmc_counters.py --timed 4 --kernel k_pull_young $R/gpurun_out/r5l_pmc/run_counter_collection.csv
cd $R
bash tools/ab/gpu_r5_c.sh
