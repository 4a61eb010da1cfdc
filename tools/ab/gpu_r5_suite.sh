# Round 5: the whole -m gpu suite (with durations) and smoke() on the final tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 1060 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread --durations=30 > gpurun_out/r5_suite.log 2>&1; rc=$?
tail -40 gpurun_out/r5_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 100 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.log 2>&1 || { tail -20 gpurun_out/r5_smoke.log; exit 1; }
tail -3 gpurun_out/r5_smoke.log
