# A/B of k_pull occupancy variants (make variants): the C4 bench once per library in $LIBS,
# loaded through GOSSIP_LIB_PATH; "base" = the default libgossip.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=p2p-gossip-simulation-ns3_amd/lib
for V in ${LIBS:-base w5 w6 q4w6 base}; do
  if [ "$V" = base ]; then P=$L/libgossip.so; else P=$L/libgossip_$V.so; fi
  GOSSIP_LIB_PATH=$PWD/$P timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/occ_$V.json 2> gpurun_out/occ_$V.err || { echo "bench [$V] failed"; tail -3 gpurun_out/occ_$V.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/occ_$V.json'));r=d['roofline'];print('[$V]', 'value %.4e ms/step %.2f pull %.3f ms bytes %.2f GB achieved %.0f GB/s frac %.4f'%(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['bytes_per_launch']/1e9,r['achieved'],r['frac']))" | tee -a gpurun_out/occ_ab.txt
done
