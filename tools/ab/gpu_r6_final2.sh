# Round 6 final evidence, part 2: every rank of the 8-GPU C4 layout rehearsed one after another
# (driver's and default arguments), the kernel trace and PMC traffic of one rank (shard 1), then the
# C3 line, trace and PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 --rehearse-index -1 > gpurun_out/r6f2_s8all.json 2> gpurun_out/r6f2_s8all.err || { tail -5 gpurun_out/r6f2_s8all.err; exit 1; }
timeout -k 10 500 python -u bench.py --steps 40 --warmup 30 --no-cpu-baseline --rehearse-shards 8 --rehearse-index -1 > gpurun_out/r6f2_s8all40.json 2> gpurun_out/r6f2_s8all40.err || { tail -5 gpurun_out/r6f2_s8all40.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r6f2_s8all.json", "gpurun_out/r6f2_s8all40.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1]); c = d["config"]
    print(f, "max", round(d["ms_per_step"], 2), [round(x, 2) for x in c["rank_ms_per_step"]], "projected %.4e" % c["projected_job_value"])
PY
cd /tmp && export TMPDIR=/tmp
B="python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --rehearse-shards 8 --rehearse-index 1"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6f2_s8trace -o run --output-format csv -- $B > $R/gpurun_out/r6f2_s8trace.json 2> $R/gpurun_out/r6f2_s8trace.err || { echo "s8 trace failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r6f2_s8pmcF -o run --output-format csv -- $B > $R/gpurun_out/r6f2_s8pmcF.json 2> $R/gpurun_out/r6f2_s8pmcF.err || { echo "s8 pmcF failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r6f2_s8pmcW -o run --output-format csv -- $B > $R/gpurun_out/r6f2_s8pmcW.json 2> $R/gpurun_out/r6f2_s8pmcW.err || { echo "s8 pmcW failed"; exit 1; }
echo s8 done
cd $R
C3="python bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline"
timeout -k 10 300 $C3 > gpurun_out/r6f2_c3.json 2> gpurun_out/r6f2_c3.err || { tail -5 gpurun_out/r6f2_c3.err; exit 1; }
python tools/ab_line.py c3 gpurun_out/r6f2_c3.json
cd /tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6f2_c3trace -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r6f2_c3trace.json 2> $R/gpurun_out/r6f2_c3trace.err || { echo "c3 trace failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc FETCH_SIZE -d $R/gpurun_out/r6f2_c3pmcF -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r6f2_c3pmcF.json 2> $R/gpurun_out/r6f2_c3pmcF.err || { echo "c3 pmcF failed"; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_pull" --pmc WRITE_SIZE -d $R/gpurun_out/r6f2_c3pmcW -o run --output-format csv -- python $R/bench.py --workload C3 --steps 40 --warmup 30 --no-cpu-baseline > $R/gpurun_out/r6f2_c3pmcW.json 2> $R/gpurun_out/r6f2_c3pmcW.err || { echo "c3 pmcW failed"; exit 1; }
echo c3 done
