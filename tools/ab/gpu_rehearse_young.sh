# N = 4 / 8 per-rank C4 workload (one GPU rehearsal): young tiles off vs on, young_age 4.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, shards, env...
    local name=$1 s=$2; shift 2
    env "$@" timeout -k 10 400 python bench.py --gpus $s --rehearse-shards $s --steps 20 --warmup 5 --no-cpu-baseline \
        > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "$name failed"; tail -3 gpurun_out/ab_$name.err; exit 1; }
    python tools/ab_line.py $name gpurun_out/ab_$name.json
}
run r8_young0 8 GOSSIP_YOUNG=0
run r8_age4 8 GOSSIP_YOUNG_AGE=4
run r4_young0 4 GOSSIP_YOUNG=0
