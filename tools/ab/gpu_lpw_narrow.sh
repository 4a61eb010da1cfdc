# 16 vs 32 word-lanes on the narrower per-rank C4 windows (N=8: 320 words, N=4: 608 words)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for S in 8 4; do
  for V in 16 32; do
    GOSSIP_PULL_LPW=$V timeout -k 10 300 python bench.py --no-cpu-baseline --rehearse-shards $S > gpurun_out/lpwn_${S}_$V.json 2> gpurun_out/lpwn_${S}_$V.err || { echo "bench [$S $V] failed"; tail -3 gpurun_out/lpwn_${S}_$V.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/lpwn_${S}_$V.json'));r=d['roofline'];print('[shards=$S lpw=$V]', 'value %.4e pull %.3f ms achieved %.0f GB/s'%(d['value'],r['avg_launch_ms'],r['achieved']))" | tee -a gpurun_out/lpw_narrow.txt
  done
done
