# Young-tile auto rule (expected slot entries per node): C4 GPU tests, the driver's bench line,
# and the N = 8 per-rank rehearsal (young tiles now off there).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 700 python -u -m pytest tests/test_scale_gpu.py -x -v --timeout 400 --timeout-method thread -m gpu > gpurun_out/gpu_scale.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_scale.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_auto.json 2> gpurun_out/bench_auto.err || { echo "bench failed"; tail -3 gpurun_out/bench_auto.err; exit 1; }
python tools/ab_line.py bench_auto gpurun_out/bench_auto.json
timeout -k 10 400 python bench.py --gpus 8 --rehearse-shards 8 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/rehearse8_auto.json 2> gpurun_out/rehearse8_auto.err || { echo "rehearse failed"; exit 1; }
python tools/ab_line.py rehearse8_auto gpurun_out/rehearse8_auto.json
