# Round 5: k_pull_young's instruction counts per segment of its node loop -- the C4 line under one
# PMC pass (SQ_INSTS_VALU / LDS / SALU, SQ_WAVES) per build: the product build and the YOUNG_DUP=k
# measurement builds (lib/yd_k: segment k run twice on the same data, same outputs); the count
# difference per launch is segment k's cost.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
L=$R/p2p-gossip-simulation-ns3_amd/lib
for v in base 1 2 3 4 5 6 7; do
  lib=$L/libgossip.so; [ $v != base ] && lib=$L/yd_$v/libgossip.so
  GOSSIP_LIB_PATH=$lib timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull_young" --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES -d $R/gpurun_out/r5i_$v -o run --output-format csv -- python $R/bench.py --steps 4 --warmup 4 --no-cpu-baseline > $R/gpurun_out/r5i_$v.json 2> $R/gpurun_out/r5i_$v.err || { echo "pmc $v failed"; tail -3 $R/gpurun_out/r5i_$v.err; exit 1; }
  echo "== $v"; python $R/tools/pmc_counters.py --timed 4 --kernel k_pull_young $R/gpurun_out/r5i_$v/run_counter_collection.csv
done
