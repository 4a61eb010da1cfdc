# Round 4: one rank of the 4- and 8-GPU C4 layouts (share shard 0 of 4 / 8 on one GPU; young tiles
# auto and forced on), the C3 line, and the BASELINE-configuration tests (C4 vs ORACLE A / B).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for s in 4 8; do
  timeout -k 10 300 python bench.py --rehearse-shards $s --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4c_s$s.json 2> gpurun_out/r4c_s$s.err || { tail -5 gpurun_out/r4c_s$s.err; exit 1; }
  python tools/ab_line.py s$s gpurun_out/r4c_s$s.json
done
GOSSIP_YOUNG=1 timeout -k 10 300 python bench.py --rehearse-shards 8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4c_s8y.json 2> gpurun_out/r4c_s8y.err || { tail -5 gpurun_out/r4c_s8y.err; exit 1; }
python tools/ab_line.py s8_young gpurun_out/r4c_s8y.json
timeout -k 10 300 python bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > gpurun_out/r4c_c3.json 2> gpurun_out/r4c_c3.err || { tail -5 gpurun_out/r4c_c3.err; exit 1; }
python tools/ab_line.py c3 gpurun_out/r4c_c3.json
timeout -k 10 700 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_scale_gpu.py -k "c4" > gpurun_out/r4c_scale.log 2>&1 || { tail -30 gpurun_out/r4c_scale.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/r4c_scale.log | tail -5
