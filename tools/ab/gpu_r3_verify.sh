# Round 3: the driver's round-end checks on the final tree -- the whole -m gpu suite (with
# durations) and smoke().
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --durations=25 --timeout 300 --timeout-method thread > gpurun_out/r3v_suite.log 2>&1
rc=$?; tail -30 gpurun_out/r3v_suite.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3v_smoke.log 2>&1 || { tail -5 gpurun_out/r3v_smoke.log; exit 1; }
tail -2 gpurun_out/r3v_smoke.log
