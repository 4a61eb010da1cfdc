# A/B of the concurrent pull phase with the early exit on: k_pull_young grid and launch order.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "$name failed"; tail -3 gpurun_out/ab_$name.err; exit 1; }
    python tools/ab_line.py $name gpurun_out/ab_$name.json
}
run ygrid2k GOSSIP_YOUNG_GRID=2048
run ygrid8k GOSSIP_YOUNG_GRID=8192
run overlap2 GOSSIP_YOUNG_OVERLAP=2
# C3 (1M nodes, below the young tiles' n >= 2^20 gate): young tiles forced on vs auto (off)
for y in -1 1; do
    GOSSIP_YOUNG=$y timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --workload C3 \
        > gpurun_out/ab_c3_young$y.json 2> gpurun_out/ab_c3_young$y.err || { echo "c3 young $y failed"; exit 1; }
    python tools/ab_line.py c3_young$y gpurun_out/ab_c3_young$y.json
done
