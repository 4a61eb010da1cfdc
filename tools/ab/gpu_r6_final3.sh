# Round 6 final evidence, part 3: the C2 (hop-batched) / C5 lines of the fused DENSE kernel and their
# rocprofv3 traces (tools/dense_trace.py), then the C5 8-rank row partition through k_dense_fused (FT
# slice exchange) and the same partition on the three-kernel path (its round-5 layout).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for c in c2 c5; do
  a="$c"; [ $c = c2 ] && a="c2 --batch"
  timeout -k 10 400 python tools/bench_dense.py $a --modes dense > gpurun_out/r6f3_$c.json 2> gpurun_out/r6f3_$c.err || { tail -5 gpurun_out/r6f3_$c.err; exit 1; }
  python tools/ab_dense.py $c gpurun_out/r6f3_$c.json
done
cd /tmp && export TMPDIR=/tmp
for c in c2 c5; do
  a="$c"; [ $c = c2 ] && a="c2 --batch"
  timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r6f3_${c}trace -o run --output-format csv -- python $R/tools/bench_dense.py $a --modes dense > $R/gpurun_out/r6f3_${c}trace.json 2> $R/gpurun_out/r6f3_${c}trace.err || { echo "$c trace failed"; tail -3 $R/gpurun_out/r6f3_${c}trace.err; exit 1; }
  python $R/tools/dense_trace.py $R/gpurun_out/r6f3_${c}trace/run_kernel_trace.csv $R/gpurun_out/r6f3_${c}trace.json > $R/gpurun_out/r6f3_${c}_span.json && grep mfma_util $R/gpurun_out/r6f3_${c}_span.json
done
cd $R
timeout -k 10 300 python -u tools/bench_dense.py c5 --row-shards 8 > gpurun_out/r6f3_c5_rows8.json 2> gpurun_out/r6f3_c5_rows8.err || { tail -5 gpurun_out/r6f3_c5_rows8.err; exit 1; }
timeout -k 10 300 python -u tools/bench_dense.py c5 --row-shards 8 --three-kernels > gpurun_out/r6f3_c5_rows8_3k.json 2> gpurun_out/r6f3_c5_rows8_3k.err || { tail -5 gpurun_out/r6f3_c5_rows8_3k.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r6f3_c5_rows8.json", "gpurun_out/r6f3_c5_rows8_3k.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, "fused", d["every_tick_fused_on_every_rank"], "phase max %.4f" % d["per_rank_phase_ms_max"], "util min %.3f" % d["per_rank_phase_util_min"],
          "bytes recv/tick %.3e" % max(d["exchange_bytes_received_per_tick_per_rank"]), "projected %.3e" % d["projected_edge_events_per_s_unmeasured"])
PY
