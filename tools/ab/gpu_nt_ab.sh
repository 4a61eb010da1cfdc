# Non-temporal row accesses on/off with the 32-lane pull: C4 (97 GB bitmaps) and C3 (2 GB).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for W in C4 C3; do
  for NT in 0 1; do
    GOSSIP_PULL_NT=$NT timeout -k 10 300 python bench.py --no-cpu-baseline --workload $W > gpurun_out/nt_${W}_$NT.json 2> gpurun_out/nt_${W}_$NT.err || { echo "bench [$W NT=$NT] failed"; tail -3 gpurun_out/nt_${W}_$NT.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/nt_${W}_$NT.json'));r=d['roofline'];print('[$W NT=$NT]', 'value %.4e pull %.3f ms achieved %.0f GB/s'%(d['value'],r['avg_launch_ms'],r['achieved']))" | tee -a gpurun_out/nt_ab_lpw32.txt
  done
done
