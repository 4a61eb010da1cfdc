# Round 5 final evidence, part 1: the shard-fallback and fused DENSE parity tests, the C2 / C5 lines and their
# rocprofv3 traces (profiles/r05/dense_*), then the C3 line, trace and PMC passes (profiles/pmc_C3.json).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest tests/test_shards_gpu.py tests/test_dense_fused_gpu.py tests/test_hop_batch.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5z1_tests.log 2>&1 || { tail -40 gpurun_out/r5z1_tests.log; exit 1; }
tail -1 gpurun_out/r5z1_tests.log
for c in c2 c5; do
  a="$c"; [ $c = c2 ] && a="c2 --batch"
  timeout -k 10 400 python tools/bench_dense.py $a --modes dense > gpurun_out/r5z1_$c.json 2> gpurun_out/r5z1_$c.err || { tail -5 gpurun_out/r5z1_$c.err; exit 1; }
  python tools/ab_dense.py $c gpurun_out/r5z1_$c.json
done
cd /tmp && export TMPDIR=/tmp
for c in c2 c5; do
  a="$c"; [ $c = c2 ] && a="c2 --batch"
  timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5z1_${c}trace -o run --output-format csv -- python $R/tools/bench_dense.py $a --modes dense > $R/gpurun_out/r5z1_${c}trace.json 2> $R/gpurun_out/r5z1_${c}trace.err || { echo "$c trace failed"; tail -3 $R/gpurun_out/r5z1_${c}trace.err; exit 1; }
  python $R/tools/dense_trace.py $R/gpurun_out/r5z1_${c}trace/run_kernel_trace.csv $R/gpurun_out/r5z1_${c}trace.json | grep mfma_util
done
cd $R
C3="python bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline"
timeout -k 10 300 $C3 > gpurun_out/r5z1_c3.json 2> gpurun_out/r5z1_c3.err || { tail -5 gpurun_out/r5z1_c3.err; exit 1; }
python tools/ab_line.py c3 gpurun_out/r5z1_c3.json
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r5z1_c3trace -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r5z1_c3trace.json 2> $R/gpurun_out/r5z1_c3trace.err || { echo "c3 trace failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r5z1_c3pmcF -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r5z1_c3pmcF.json 2> $R/gpurun_out/r5z1_c3pmcF.err || { echo "c3 pmcF failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r5z1_c3pmcW -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r5z1_c3pmcW.json 2> $R/gpurun_out/r5z1_c3pmcW.err || { echo "c3 pmcW failed"; exit 1; }
echo c3 done
