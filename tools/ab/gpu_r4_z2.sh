# Round 4 evidence, part 2 (final tree): C3 line + trace + PMC passes, one rank of the 4- and
# 8-GPU C4 layouts (rehearsals), the dense C2 / C5 lines (one event pair around the DENSE phase)
# and the C2 trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
C3="python bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline"
timeout -k 10 300 $C3 > gpurun_out/r4z_c3.json 2> gpurun_out/r4z_c3.err || { tail -5 gpurun_out/r4z_c3.err; exit 1; }
python tools/ab_line.py c3 gpurun_out/r4z_c3.json
for s in 4 8; do
  timeout -k 10 300 python bench.py --rehearse-shards $s --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r4z_s$s.json 2> gpurun_out/r4z_s$s.err || { tail -5 gpurun_out/r4z_s$s.err; exit 1; }
  python tools/ab_line.py s$s gpurun_out/r4z_s$s.json
done
timeout -k 10 300 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/r4z_c2.json 2> gpurun_out/r4z_c2.err || { tail -5 gpurun_out/r4z_c2.err; exit 1; }
cat gpurun_out/r4z_c2.json
timeout -k 10 300 python tools/bench_dense.py c5 --modes dense > gpurun_out/r4z_c5.json 2> gpurun_out/r4z_c5.err || { tail -5 gpurun_out/r4z_c5.err; exit 1; }
cat gpurun_out/r4z_c5.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4z_c3trace -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r4z_c3trace.json 2> $R/gpurun_out/r4z_c3trace.err || { echo "c3 trace failed"; tail -3 $R/gpurun_out/r4z_c3trace.err; exit 1; }
echo c3 trace ok
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r4z_c3pmcF -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r4z_c3pmcF.json 2> $R/gpurun_out/r4z_c3pmcF.err || { echo "c3 pmcF failed"; tail -3 $R/gpurun_out/r4z_c3pmcF.err; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r4z_c3pmcW -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r4z_c3pmcW.json 2> $R/gpurun_out/r4z_c3pmcW.err || { echo "c3 pmcW failed"; tail -3 $R/gpurun_out/r4z_c3pmcW.err; exit 1; }
echo c3 pmc ok
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4z_c2trace -o run --output-format csv -- python $R/tools/bench_dense.py c2 --batch --modes dense > $R/gpurun_out/r4z_c2trace.json 2> $R/gpurun_out/r4z_c2trace.err || { echo "c2 trace failed"; tail -3 $R/gpurun_out/r4z_c2trace.err; exit 1; }
echo c2 trace ok
