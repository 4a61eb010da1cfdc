# A/B of the late-tile early exit (option late_age, env GOSSIP_LATE_AGE) on C4, driver command
# shape; then the parity tests of the option.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
B="python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 400 $B > gpurun_out/ab_$name.json 2> gpurun_out/ab_$name.err || { echo "$name failed"; tail -3 gpurun_out/ab_$name.err; exit 1; }
    python tools/ab_line.py $name gpurun_out/ab_$name.json
}
for a in ${LATE_AGES:-0 8 7 9}; do
    run late$a GOSSIP_LATE_AGE=$a
done
timeout -k 10 600 python -u -m pytest tests/test_late_exit_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/gpu_late.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_late.log; [ $rc -eq 0 ] || exit 1
