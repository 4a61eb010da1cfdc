# Sparse pull lanes-per-node A/B: GPU suite with every wide window forced onto 32 lanes
# (parity of the k_pull<32,1> wide path), then the N=8 per-rank C4 workload (320 words/node)
# with the automatic rule (-> 32 lanes) and forced 64 lanes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
GOSSIP_PULL_LPW=32 timeout -k 10 400 python -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/gpu_tests_lpw32.log 2>&1
rc=$?; echo "pytest (LPW=32) rc=$rc"; tail -2 gpurun_out/gpu_tests_lpw32.log; [ $rc -eq 0 ] || exit 1
for V in auto 64 auto; do
  if [ $V = auto ]; then E=""; else E="GOSSIP_PULL_LPW=$V"; fi
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --rehearse-shards 8 > gpurun_out/lpw_$V.json 2> gpurun_out/lpw_$V.err || { echo "bench [$V] failed"; tail -3 gpurun_out/lpw_$V.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/lpw_$V.json'));r=d['roofline'];print('[s8 lpw=$V]', 'value %.4e pull %.3f ms achieved %.0f GB/s'%(d['value'],r['avg_launch_ms'],r['achieved']))" | tee -a gpurun_out/lpw_ab.txt
done
