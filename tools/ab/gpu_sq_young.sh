# SQ instruction/stall counters for k_pull and k_pull_young on one C4 shard (rehearsal of shard 0
# of 2, 5 timed ticks); one counter pass, kernels filtered to the pulls.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-include-regex "k_pull_young" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY -d $R/gpurun_out/sq_young -o run --output-format csv -- python $R/bench.py --rehearse-shards 2 --steps 5 --warmup 5 --no-cpu-baseline > $R/gpurun_out/sq_young.json 2> $R/gpurun_out/sq_young.err || { echo "sq pass failed"; tail -5 $R/gpurun_out/sq_young.err; exit 1; }
echo sq done
