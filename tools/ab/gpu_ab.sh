# A/B iteration: GPU parity suite, then the C3 bench once per argument set in $VARIANTS
# (separated by ';', e.g. VARIANTS="--pull-kernel auto;--pull-kernel generic").
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit 1
IFS=';' read -ra VS <<< "${VARIANTS:- }"
i=0
for V in "${VS[@]}"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --no-cpu-baseline $V > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { echo "bench [$V] failed"; tail -3 gpurun_out/ab_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$i.json'));r=d['roofline'];print('[$V]', 'value %.3e ms/step %.3f pull %.3f ms bytes %.2f GB achieved %.0f GB/s frac %.3f'%(d['value'],d['ms_per_step'],r['avg_launch_ms'],r['bytes_per_launch']/1e9,r['achieved'],r['frac']))"
done
