# Round 6: the MFMA pipe's busy cycles and the shader clock of k_dense_fused by PMC (one pass:
# SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE) on C5 and C2 hop-batched -- the counter
# view of DESIGN §6's stamp breakdown.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for c in c5 c2; do
  a="$c"; [ $c = c2 ] && a="c2 --batch"
  timeout -s KILL 240 rocprofv3 --kernel-include-regex "k_dense_fused" --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/r6r_$c -o run --output-format csv -- python $R/tools/bench_dense.py $a --modes dense > $R/gpurun_out/r6r_$c.json 2> $R/gpurun_out/r6r_$c.err || { echo "$c pmc failed"; tail -5 $R/gpurun_out/r6r_$c.err; exit 1; }
  ls $R/gpurun_out/r6r_$c
done
