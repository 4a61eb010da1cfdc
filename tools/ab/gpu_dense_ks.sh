# Dense split-K target (GOSSIP_DENSE_MIN_TILES) A/B on hop-batched C2 and the C5 4096-share slice.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for T in 512 1024 2048 256 512; do
  for R in 1 2; do
    GOSSIP_DENSE_MIN_TILES=$T timeout -k 10 200 python -u tools/bench_dense.py c2 --batch --modes dense > gpurun_out/ks_c2_$T.json 2> gpurun_out/ks_c2_$T.err || { echo c2 failed; tail -3 gpurun_out/ks_c2_$T.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ks_c2_$T.json').read().splitlines()[-1]);print('[C2 batch tiles=$T]', 'mfma %.3f ms util %.3f'%(d['pull_ms_avg'], d['mfma_util']))" | tee -a gpurun_out/ks_ab.txt
  done
done
for T in 512 1024 2048; do
  GOSSIP_DENSE_MIN_TILES=$T timeout -k 10 300 python -u tools/bench_dense.py c5 --width 4096 --modes dense > gpurun_out/ks_c5_$T.json 2> gpurun_out/ks_c5_$T.err || { echo c5 failed; tail -3 gpurun_out/ks_c5_$T.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ks_c5_$T.json').read().splitlines()[-1]);print('[C5 w4096 tiles=$T]', 'mfma %.3f ms util %.3f'%(d['pull_ms_avg'], d['mfma_util']))" | tee -a gpurun_out/ks_ab.txt
done
