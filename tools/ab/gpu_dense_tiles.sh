# C2 (hop-batched) with 1024-k stages: the K-split target (dense_min_tiles).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for t in 256 512 1024; do
    GOSSIP_DENSE_MIN_TILES=$t timeout -k 10 200 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/dt_c2_$t.json 2> gpurun_out/dt_c2_$t.err || { echo "tiles $t failed"; exit 1; }
    python -c "
import json
d=[json.loads(l) for l in open('gpurun_out/dt_c2_$t.json') if l.startswith('{')][-1]
print('[c2 tiles=$t]', {k: d[k] for k in d if 'util' in k or 'ms_avg' in k})"
done
