# Round 3 final kernels: SQ counters of k_pull and k_pull_young on one C4 shard (one PMC pass; the
# profiler serialises the kernels), to compare with profiles/r03/c4_sq_counters.json (r02 kernels).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD -d $R/gpurun_out/r3f_sq -o run --output-format csv -- python $R/bench.py --rehearse-shards 2 --steps 5 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r3f_sq.json 2> $R/gpurun_out/r3f_sq.err || { echo "sq failed"; tail -3 $R/gpurun_out/r3f_sq.err; exit 1; }
for k in "k_pull<32" "k_pull_young"; do echo "$k"; python $R/tools/pmc_counters.py --timed 5 --kernel "$k" $R/gpurun_out/r3f_sq/run_counter_collection.csv; done
