# Second A/B of the late-tile early exit: every tile on C4, and C3 (no young tiles) at several ages.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {  # name, workload, env...
    local name=$1 wl=$2; shift 2
    env "$@" timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --workload $wl \
        > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "$name failed"; tail -3 gpurun_out/ab_$name.err; exit 1; }
    python tools/ab_line.py $name gpurun_out/ab_$name.json
}
for a in 0 4 5 6 1; do run c3_late$a C3 GOSSIP_LATE_AGE=$a; done
run c4_late1 C4 GOSSIP_LATE_AGE=1
timeout -k 10 600 python -u -m pytest tests/test_late_exit_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/gpu_late.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_late.log; [ $rc -eq 0 ] || exit 1
