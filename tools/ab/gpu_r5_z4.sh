# Round 5: one rank of 4 shards (the N = 4 layout): hash rule packed (the default) vs hash with a
# fresh tile per tick vs the tick rule (fresh tiles), twice each, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 4 "$@" > gpurun_out/r5z4_$name.json 2> gpurun_out/r5z4_$name.err || { tail -5 gpurun_out/r5z4_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r5z4_$name.json
}
for rep in 1 2; do
  run hash$rep
  run hashfresh$rep --fresh-tiles on
  run tick$rep --shard-rule tick
done
