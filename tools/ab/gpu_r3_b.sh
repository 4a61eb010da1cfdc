# Round 3, call B: the gate fix under the C3 tests and the wide-peer-list regression test; the
# DENSE dedup kernel's SQ counters (why ~150 us per C2 dispatch?); available counters.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest tests/test_c3_gpu.py tests/test_late_exit_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread --durations=0 > gpurun_out/r3_tests_b.log 2>&1
rc=$?; tail -25 gpurun_out/r3_tests_b.log; [ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $R/gpurun_out/r3_counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_dense_dedup|k_dense_bits" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $R/gpurun_out/r3_dedup_pmc -o run --output-format csv -- python $R/tools/bench_dense.py c2 --batch --modes dense > $R/gpurun_out/r3_dedup_pmc.json 2> $R/gpurun_out/r3_dedup_pmc.err || { echo "pmc failed"; tail -3 $R/gpurun_out/r3_dedup_pmc.err; exit 1; }
echo pmc ok
