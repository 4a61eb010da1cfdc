# A/B of k_pull_young's seen-row touch (option young_touch) on C4, driver command shape.
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
run touch0 GOSSIP_YOUNG_TOUCH=0
run touch1 GOSSIP_YOUNG_TOUCH=1
run touch1_seq GOSSIP_YOUNG_TOUCH=1 GOSSIP_YOUNG_OVERLAP=0
