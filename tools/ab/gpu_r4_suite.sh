# Round 4: the whole -m gpu suite and smoke() on the final tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r4_suite.log 2>&1; rc=$?
tail -5 gpurun_out/r4_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.log 2>&1 || { tail -20 gpurun_out/r4_smoke.log; exit 1; }
tail -3 gpurun_out/r4_smoke.log
