# Round 4: k_pull_young's young_age (tiles of hops <= age in slots) re-measured with the round-4
# kernels on the driver's bench arguments, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4s_$name.json 2> gpurun_out/r4s_$name.err || { tail -5 gpurun_out/r4s_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4s_$name.json
}
run now
run age4 GOSSIP_YOUNG_AGE=4
run age6 GOSSIP_YOUNG_AGE=6
run now2
