# Round 6: the whole -m gpu suite (with durations) and smoke() on the current tree, then the C5
# 8-rank row-partition rehearsal (fused ranks, FT slice exchange).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 1060 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread --durations=40 > gpurun_out/r6_suite.log 2>&1; rc=$?
tail -50 gpurun_out/r6_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.log 2>&1 || { tail -20 gpurun_out/r6_smoke.log; exit 1; }
tail -3 gpurun_out/r6_smoke.log
timeout -k 10 300 python -u tools/bench_dense.py c5 --row-shards 8 > gpurun_out/r6_c5_rows8.json 2> gpurun_out/r6_c5_rows8.err || { tail -5 gpurun_out/r6_c5_rows8.err; exit 1; }
tail -c 2500 gpurun_out/r6_c5_rows8.json
