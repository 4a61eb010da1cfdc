# Round 4 baseline on this round's boxes: the driver's bench command (C4, N = 1) on the r03 tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4_base.json 2> gpurun_out/r4_base.err || { tail -5 gpurun_out/r4_base.err; exit 1; }
python tools/ab_line.py base gpurun_out/r4_base.json
