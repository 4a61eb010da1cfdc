# Per-rank workload of the N=8 C4 run (shard 0 of 8 on one GPU) under each pull kernel.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for K in ${KERNELS:-auto wide generic}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --rehearse-shards 8 --pull-kernel $K ${BENCH_ARGS:-} > gpurun_out/s8_$K.json 2> gpurun_out/s8_$K.err || { echo "bench [$K] failed"; tail -3 gpurun_out/s8_$K.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/s8_$K.json'));r=d['roofline'];print('[$K]', 'value %.4e pull %.3f ms bytes %.2f GB achieved %.0f GB/s'%(d['value'],r['avg_launch_ms'],r['bytes_per_launch']/1e9,r['achieved']), {k: round(v/1e9,2) for k,v in r['bytes_breakdown_per_launch'].items()}, d['config'].get('live_words_per_node'))" | tee -a gpurun_out/s8_ab.txt
done
