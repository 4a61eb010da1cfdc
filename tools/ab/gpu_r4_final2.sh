# Round 4 final tree (young grid 2x the pull grid): the whole -m gpu suite with durations, smoke(),
# the driver's bench command with its CPU baselines, and the rocprofv3 kernel trace + stats of the
# same command (PMC traffic: the pmc_C4*.json passes of gpu_r4_z1.sh, same kernels and config).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread --durations=25 > gpurun_out/r4g2_suite.log 2>&1; rc=$?
tail -30 gpurun_out/r4g2_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4g2_smoke.log 2>&1 || { tail -20 gpurun_out/r4g2_smoke.log; exit 1; }
tail -2 gpurun_out/r4g2_smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4g2_bench.json 2> gpurun_out/r4g2_bench.err || { tail -5 gpurun_out/r4g2_bench.err; exit 1; }
python tools/ab_line.py final gpurun_out/r4g2_bench.json
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4g2_trace -o run --output-format csv -- $B > $R/gpurun_out/r4g2_trace.json 2> $R/gpurun_out/r4g2_trace.err || { echo "trace failed"; tail -3 $R/gpurun_out/r4g2_trace.err; exit 1; }
echo trace ok
