# 16 vs 32 word-lanes per node: C4 N=1 (1216 words) and C3 (1M nodes, 118 words)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for W in C4 C3; do
  for V in 32 16 64; do
    GOSSIP_PULL_LPW=$V timeout -k 10 300 python bench.py --no-cpu-baseline --workload $W > gpurun_out/lpw3_${W}_$V.json 2> gpurun_out/lpw3_${W}_$V.err || { echo "bench [$W $V] failed"; tail -3 gpurun_out/lpw3_${W}_$V.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/lpw3_${W}_$V.json'));r=d['roofline'];print('[$W lpw=$V]', 'value %.4e pull %.3f ms achieved %.0f GB/s words %s'%(d['value'],r['avg_launch_ms'],r['achieved'],d['config'].get('live_words_per_node')))" | tee -a gpurun_out/lpw_ab3.txt
  done
done
