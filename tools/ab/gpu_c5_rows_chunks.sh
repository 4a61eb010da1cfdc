# C5 row partition x8 rehearsed on one GPU (lockstep group): per-rank MFMA time with the
# exchange in 1 vs 4 row chunks (the pipelined exchange's compute-side cost).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for x in 1 4; do
    GOSSIP_XCHUNKS=$x timeout -k 10 300 python tools/bench_dense.py c5 --width 4096 --row-shards 8 --modes dense \
        > gpurun_out/c5_rows_x$x.json 2> gpurun_out/c5_rows_x$x.err || { echo "x$x failed"; tail -3 gpurun_out/c5_rows_x$x.err; exit 1; }
    echo "xchunks=$x"; tail -1 gpurun_out/c5_rows_x$x.json
done
