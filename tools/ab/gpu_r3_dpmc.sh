# Round 3: dense (int8 MFMA) path on the final tree: kernel trace + stats and an
# SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE pass of k_dense_bits on C2 (hop-batched, 60 s) and the
# C5 flood (4,096 shares) -- as tools/ab/gpu_prof_dense.sh did for round 2.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in "c2 --batch" "c5 --width 4096"; do
  tag=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r3d_$tag -o run --output-format csv -- python $R/tools/bench_dense.py $C --modes dense > $R/gpurun_out/r3d_$tag.json 2> $R/gpurun_out/r3d_$tag.err || { echo "trace $tag failed"; tail -3 $R/gpurun_out/r3d_$tag.err; exit 1; }
  timeout -s KILL 300 rocprofv3 --kernel-include-regex "k_dense_bits" --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $R/gpurun_out/r3d_pmc_$tag -o run --output-format csv -- python $R/tools/bench_dense.py $C --modes dense > $R/gpurun_out/r3d_pmc_$tag.json 2> $R/gpurun_out/r3d_pmc_$tag.err || { echo "pmc $tag failed"; tail -3 $R/gpurun_out/r3d_pmc_$tag.err; exit 1; }
  echo "$tag ok"
done
