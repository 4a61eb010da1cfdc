# Round 3: the whole -m gpu suite as the driver runs it, with per-test durations (suite budget).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 1100 python -u -m pytest tests/ -m gpu -x -q --durations=0 --timeout 300 --timeout-method thread > gpurun_out/r3s_suite.log 2>&1
rc=$?; tail -60 gpurun_out/r3s_suite.log; exit $rc
