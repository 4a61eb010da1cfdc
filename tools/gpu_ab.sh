# A/B iteration: GPU parity suite on the default library, then the C3 bench for each library
# named in $LIBS (paths relative to the package lib/ directory).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit 1
for L in ${LIBS:-libgossip.so}; do
  GOSSIP_LIB_PATH=$GRAFT_REPO_ROOT/p2p-gossip-simulation-ns3_amd/lib/$L timeout -k 10 200 python bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/ab_$L.json 2> gpurun_out/ab_$L.err || { echo "bench $L failed"; tail -3 gpurun_out/ab_$L.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$L.json'));r=d['roofline'];print('$L', 'value %.3e ms/step %.3f pull %.3f ms bytes %.2f GB achieved %.0f GB/s frac %.3f'%(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['bytes_per_launch']/1e9,r['achieved'],r['frac']))"
done
