# 32 vs 64 word-lanes per node at the other C4 per-rank widths: N=1 (1232 words), N=4 (608).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for S in 1 4; do
  for V in 64 32; do
    if [ $S = 1 ]; then A=""; else A="--rehearse-shards $S"; fi
    GOSSIP_PULL_LPW=$V timeout -k 10 300 python bench.py --no-cpu-baseline $A > gpurun_out/lpw2_${S}_$V.json 2> gpurun_out/lpw2_${S}_$V.err || { echo "bench [$S $V] failed"; tail -3 gpurun_out/lpw2_${S}_$V.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/lpw2_${S}_$V.json'));r=d['roofline'];print('[shards=$S lpw=$V]', 'value %.4e pull %.3f ms achieved %.0f GB/s words %s'%(d['value'],r['avg_launch_ms'],r['achieved'],d['config'].get('live_words_per_node')))" | tee -a gpurun_out/lpw_ab2.txt
  done
done
