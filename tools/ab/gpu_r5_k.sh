# Round 5: k_pull_young with the merged entry loop (64 VGPRs again) and k_dense_fused at GM = 4:
# young + C4 parity, the fused DENSE tests, then a same-box A/B of the C4 line against the
# round-4 kernels (lib/var_tl: commit fceb2f7), and one PMC pass of k_pull_young's instructions.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_young_gpu.py tests/test_late_exit_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5k_young_tests.log 2>&1 || { tail -40 gpurun_out/r5k_young_tests.log; exit 1; }
tail -1 gpurun_out/r5k_young_tests.log
timeout -k 10 700 python -u -m pytest tests/test_scale_gpu.py -k "c4" -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/r5k_c4_tests.log 2>&1 || { tail -40 gpurun_out/r5k_c4_tests.log; exit 1; }
tail -1 gpurun_out/r5k_c4_tests.log
timeout -k 10 400 python -u -m pytest tests/test_dense_fused_gpu.py -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/r5k_fused_tests.log 2>&1 || { tail -40 gpurun_out/r5k_fused_tests.log; exit 1; }
tail -1 gpurun_out/r5k_fused_tests.log
L=$R/p2p-gossip-simulation-ns3_amd/lib
for rep in 1 2; do
  for v in cur r4; do
    lib=$L/libgossip.so; [ $v = r4 ] && lib=$L/var_tl/libgossip.so
    GOSSIP_LIB_PATH=$lib timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r5k_${v}$rep.json 2> gpurun_out/r5k_${v}$rep.err || { tail -5 gpurun_out/r5k_${v}$rep.err; exit 1; }
    python tools/ab_line.py ${v}$rep gpurun_out/r5k_${v}$rep.json
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull_young" --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/r5k_pmc -o run --output-format csv -- python $R/bench.py --steps 4 --warmup 4 --no-cpu-baseline > $R/gpurun_out/r5k_pmc.json 2> $R/gpurun_out/r5k_pmc.err || { echo "pmc failed"; tail -3 $R/gpurun_out/r5k_pmc.err; exit 1; }
python $R/tools/pmc_counters.py --timed 4 --kernel k_pull_young $R/gpurun_out/r5k_pmc/run_counter_collection.csv
