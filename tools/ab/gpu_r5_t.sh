# Round 5: the two pull kernels one after the other (young_overlap 0: k_pull alone, k_pull_young
# alone, same run) on the C4 line and on one rank of 8 shards; then the 8-shard rank's PMC traffic
# passes (FETCH_SIZE, WRITE_SIZE; both pull kernels, tools/pmc_traffic.py afterwards on the CPU).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, bench args..., then env after --
  local name=$1; shift
  env GOSSIP_YOUNG_OVERLAP=0 timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/r5t_$name.json 2> gpurun_out/r5t_$name.err || { tail -5 gpurun_out/r5t_$name.err; exit 1; }
  python tools/ab_line.py $name gpurun_out/r5t_$name.json
}
run c4_seq
run s8_seq --rehearse-shards 8
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8"
timeout -k 10 300 $B > $R/gpurun_out/r5t_s8_line.json 2> $R/gpurun_out/r5t_s8_line.err || { echo "s8 line failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r5t_s8_pmcF -o run --output-format csv -- $B > $R/gpurun_out/r5t_s8_pmcF.json 2> $R/gpurun_out/r5t_s8_pmcF.err || { echo "pmcF failed"; tail -3 $R/gpurun_out/r5t_s8_pmcF.err; exit 1; }
echo pmcF ok
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r5t_s8_pmcW -o run --output-format csv -- $B > $R/gpurun_out/r5t_s8_pmcW.json 2> $R/gpurun_out/r5t_s8_pmcW.err || { echo "pmcW failed"; tail -3 $R/gpurun_out/r5t_s8_pmcW.err; exit 1; }
echo pmcW ok
