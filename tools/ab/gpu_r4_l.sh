# Round 4: launch knobs on the final kernels (env-var engine options, one box): k_pull lanes per
# node 64 (8 tiles per pass), k_pull grid 8k / 32k blocks, k_pull_young grid 4k / 32k blocks, and
# k_pull capped at 4 blocks per CU by reserved LDS (34 KB: one k_pull_young block fits beside; 36 KB: none).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 $B > gpurun_out/r4l_$name.json 2> gpurun_out/r4l_$name.err || { tail -5 gpurun_out/r4l_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r4l_$name.json
}
run now
run lpw64 GOSSIP_PULL_LPW=64
run grid8k GOSSIP_PULL_GRID=8192
run grid32k GOSSIP_PULL_GRID=32768
run ygrid4k GOSSIP_YOUNG_GRID=4096
run ygrid32k GOSSIP_YOUNG_GRID=32768
run lds34k GOSSIP_PULL_LDS_MIN=34816
run lds36k GOSSIP_PULL_LDS_MIN=36864
run lds34k_seq GOSSIP_PULL_LDS_MIN=34816 GOSSIP_YOUNG_OVERLAP=0
# one rank of the 8-GPU layout with young tiles forced on (auto keeps them off at ~12 entries)
for y in 1; do
  GOSSIP_YOUNG=$y timeout -k 10 300 python bench.py --rehearse-shards 8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4l_s8y$y.json 2> gpurun_out/r4l_s8y$y.err || { tail -5 gpurun_out/r4l_s8y$y.err; exit 1; }
  python tools/ab_line.py s8_young$y gpurun_out/r4l_s8y$y.json
done
