# Per-rank workload of the N = 2 / 4 / 8 C4 bench lines, rehearsed on one GPU (bench.py
# --rehearse-shards S: shard 0 of S, timed like one rank), with the round-2 kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for s in 2 4 8; do
    timeout -k 10 400 python bench.py --gpus $s --rehearse-shards $s --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/rehearse$s.json 2> gpurun_out/rehearse$s.err || { echo "rehearse $s failed"; tail -3 gpurun_out/rehearse$s.err; exit 1; }
    python tools/ab_line.py rehearse$s gpurun_out/rehearse$s.json
done
