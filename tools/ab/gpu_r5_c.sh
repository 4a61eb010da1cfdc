# Round 5: birth-tick share sharding (GOSSIP_F_SHARD_BY_TICK) against the hash rule, same box:
# one rank of the 8-GPU C4 layout (shard 0 of 8, rehearsed on this GPU) and the 2-shard N = 1 line.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 500 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/r5c_$name.json 2> gpurun_out/r5c_$name.err || { tail -5 gpurun_out/r5c_$name.err; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/r5c_$name.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$name', '%.4g'%d['value'], 'ms/step %.2f'%d['ms_per_step'], 'phase %.2f'%r['avg_launch_ms'], 'frac %.3f'%r['frac'])"
}
run s8_tick --rehearse-shards 8 --shard-rule tick
run s8_hash --rehearse-shards 8 --shard-rule hash
run n1_tick --shard-rule tick
run n1_hash --shard-rule hash
