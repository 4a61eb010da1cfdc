# Round 3: the driver's bench command on the current tree (C4, N = 1), then the rocprofv3 kernel
# trace + stats of the same command.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3f_bench.json 2> gpurun_out/r3f_bench.err || { tail -5 gpurun_out/r3f_bench.err; exit 1; }
python tools/ab_line.py final gpurun_out/r3f_bench.json
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3f_trace -o run --output-format csv -- $B > $R/gpurun_out/r3f_trace.json 2> $R/gpurun_out/r3f_trace.err || { echo "trace failed"; tail -3 $R/gpurun_out/r3f_trace.err; exit 1; }
echo trace ok
