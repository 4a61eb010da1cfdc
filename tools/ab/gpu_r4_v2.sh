# Round 4, after the share-ownership host change: the whole -m gpu suite with durations,
# smoke(), and the driver's default bench command.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread --durations=25 > gpurun_out/r4v2_suite.log 2>&1; rc=$?
tail -32 gpurun_out/r4v2_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4v2_smoke.log 2>&1 || { tail -20 gpurun_out/r4v2_smoke.log; exit 1; }
tail -2 gpurun_out/r4v2_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r4v2_bench.json 2> gpurun_out/r4v2_bench.err || { tail -5 gpurun_out/r4v2_bench.err; exit 1; }
python tools/ab_line.py default gpurun_out/r4v2_bench.json
