# Round 4 final tree: the whole -m gpu suite with durations, smoke(), the driver's bench command,
# and the k_pull_young 32k-block grid against the default on the same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread --durations=25 > gpurun_out/r4f_suite.log 2>&1; rc=$?
tail -32 gpurun_out/r4f_suite.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 || { tail -20 gpurun_out/r4f_smoke.log; exit 1; }
tail -2 gpurun_out/r4f_smoke.log
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4f_$name.json 2> gpurun_out/r4f_$name.err || { tail -5 gpurun_out/r4f_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4f_$name.json
}
run now
run ygrid32k GOSSIP_YOUNG_GRID=32768
run now2
run ygrid32k_2 GOSSIP_YOUNG_GRID=32768
