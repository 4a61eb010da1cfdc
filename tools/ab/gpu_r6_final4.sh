# Round 6 final evidence, the C3 part of part 2 alone (line, trace, PMC passes) -- for a rebuilt library
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
C3="python bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline"
timeout -k 10 300 $C3 > gpurun_out/r6f2_c3.json 2> gpurun_out/r6f2_c3.err || { tail -5 gpurun_out/r6f2_c3.err; exit 1; }
python tools/ab_line.py c3 gpurun_out/r6f2_c3.json
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6f2_c3trace -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r6f2_c3trace.json 2> $R/gpurun_out/r6f2_c3trace.err || { echo "c3 trace failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r6f2_c3pmcF -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r6f2_c3pmcF.json 2> $R/gpurun_out/r6f2_c3pmcF.err || { echo "c3 pmcF failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r6f2_c3pmcW -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r6f2_c3pmcW.json 2> $R/gpurun_out/r6f2_c3pmcW.err || { echo "c3 pmcW failed"; exit 1; }
echo c3 done
bash $R/tools/ab/gpu_r6_final3.sh
