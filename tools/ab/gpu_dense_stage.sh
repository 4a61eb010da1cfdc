# A/B of the MFMA contraction's LDS stage (k per stage 512 vs 1024: half the barriers) on C2
# (hop-batched) and the C5 slice, after the dense parity tests on the 1024 build.
set -o pipefail
R=$GRAFT_REPO_ROOT
L=$R/p2p-gossip-simulation-ns3_amd/lib
mkdir -p $R/gpurun_out
cd $R
GOSSIP_LIB_PATH=$L/libgossip_dk1024.so timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_hop_batch.py tests/test_row_partition.py -x -v --timeout 300 --timeout-method thread -m gpu -k "dense or mfma or hop" > gpurun_out/gpu_dk.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/gpu_dk.log; [ $rc -eq 0 ] || exit 1
for v in base dk1024; do
    lib=$L/libgossip.so; [ $v = dk1024 ] && lib=$L/libgossip_dk1024.so
    GOSSIP_LIB_PATH=$lib timeout -k 10 200 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/dk_c2_$v.json 2> gpurun_out/dk_c2_$v.err || { echo "c2 $v failed"; exit 1; }
    GOSSIP_LIB_PATH=$lib timeout -k 10 200 python tools/bench_dense.py c5 --width 4096 --modes dense > gpurun_out/dk_c5_$v.json 2> gpurun_out/dk_c5_$v.err || { echo "c5 $v failed"; exit 1; }
    echo "== $v"; python -c "
import json,sys
for f in ['gpurun_out/dk_c2_$v.json','gpurun_out/dk_c5_$v.json']:
    d=[json.loads(l) for l in open(f) if l.startswith('{')][-1]
    print(f, {k: d[k] for k in d if 'util' in k or 'ms' in k or 'edge_events_per' in k})"
done
