# Round 5 DIAGNOSTIC (results wrong by design): the cost of k_pull's passes over old tiles.  The
# lib/var_sk build (Makefile engine_sk.o) leaves tiles at least GOSSIP_DIAG_SKIP_AGE ticks old out of
# k_pull's lists; the time it saves prices the straggler passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
L=$R/p2p-gossip-simulation-ns3_amd/lib
run() {  # name, bench args..., env via ENVS
  local name=$1; shift
  env $ENVS timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/r5x_$name.json 2> gpurun_out/r5x_$name.err || { tail -5 gpurun_out/r5x_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r5x_$name.json
}
ENVS="X=1" run s8_base --rehearse-shards 8
for a in 9 12; do ENVS="GOSSIP_LIB_PATH=$L/var_sk/libgossip.so GOSSIP_DIAG_SKIP_AGE=$a" run s8_sk$a --rehearse-shards 8; done
ENVS="X=1" run c4_base
for a in 8 10 12; do ENVS="GOSSIP_LIB_PATH=$L/var_sk/libgossip.so GOSSIP_DIAG_SKIP_AGE=$a" run c4_sk$a; done
