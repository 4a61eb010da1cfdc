# Round 3: C4 layout decision on measured numbers -- one rank of each candidate
# 8-GPU layout rehearsed on this one GPU: share shards x8 (the bench's layout), and the hybrid
# S share shards x R row ranks (2 x 4, 2 x 8, 4 x 2) through bench.py --rehearse-rows.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
A="--steps 20 --warmup 5 --no-cpu-baseline"
if [ "${WITH_S8:-0}" = 1 ]; then
timeout -k 10 420 python bench.py $A --rehearse-shards 8 > gpurun_out/r3_rows_s8.json 2> gpurun_out/r3_rows_s8.err || { tail -5 gpurun_out/r3_rows_s8.err; exit 1; }
python tools/ab_line.py s8 gpurun_out/r3_rows_s8.json
fi
for SR in "2 4" "2 8" "4 2"; do
  set -- $SR
  timeout -k 10 420 python bench.py $A --rehearse-shards $1 --rehearse-rows $2 > gpurun_out/r3_rows_s$1r$2.json 2> gpurun_out/r3_rows_s$1r$2.err || { tail -5 gpurun_out/r3_rows_s$1r$2.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r3_rows_s$1r$2.json').read().strip().splitlines()[-1])
print('S=$1 R=$2', {k: (round(v,3) if isinstance(v,float) else v) for k,v in d.items() if k in ('rank_gpu_ms_per_tick_max','rank_ingress_bytes_per_tick_max','unpartitioned_pull_ms_per_tick','rank_device_gib','window_words')})"
done
timeout -k 10 300 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/r3r_dense_c2.json 2> gpurun_out/r3r_dense_c2.err || exit 1
cat gpurun_out/r3r_dense_c2.json
