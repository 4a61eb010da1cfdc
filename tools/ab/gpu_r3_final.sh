# Round 3 final line: the driver's bench command (C4, N = 1), the rocprofv3 kernel trace + stats
# of the same command, and the C3 line with young tiles auto (off below 2^20 nodes) vs forced on.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3z_bench.json 2> gpurun_out/r3z_bench.err || { tail -5 gpurun_out/r3z_bench.err; exit 1; }
python tools/ab_line.py final gpurun_out/r3z_bench.json
for y in -1 1; do
  GOSSIP_YOUNG=$y timeout -k 10 200 python bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > gpurun_out/r3z_c3_y$y.json 2> gpurun_out/r3z_c3_y$y.err || { tail -5 gpurun_out/r3z_c3_y$y.err; exit 1; }
  python tools/ab_line.py c3_young$y gpurun_out/r3z_c3_y$y.json
done
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3z_trace -o run --output-format csv -- $B > $R/gpurun_out/r3z_trace.json 2> $R/gpurun_out/r3z_trace.err || { echo "trace failed"; tail -3 $R/gpurun_out/r3z_trace.err; exit 1; }
echo trace ok
