# Round 3: slice vs continuous discrepancy hunt (tools/diag_slice.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/r3_dense_c2b.json 2> gpurun_out/r3_dense_c2b.err && cat gpurun_out/r3_dense_c2b.json
timeout -k 10 300 python tools/diag_slice.py --nodes 200000 --variants > gpurun_out/r3_diag_200k.json 2> gpurun_out/r3_diag_200k.err || { tail -5 gpurun_out/r3_diag_200k.err; exit 1; }
cat gpurun_out/r3_diag_200k.json
timeout -k 10 300 python tools/diag_slice.py --nodes 200000 --life 40 > gpurun_out/r3_diag_200k_l40.json 2>> gpurun_out/r3_diag_200k.err || exit 1
cat gpurun_out/r3_diag_200k_l40.json
timeout -k 10 400 python tools/diag_slice.py --variants > gpurun_out/r3_diag_1m.json 2> gpurun_out/r3_diag_1m.err || { tail -5 gpurun_out/r3_diag_1m.err; exit 1; }
cat gpurun_out/r3_diag_1m.json
timeout -k 10 300 python tools/bench_dense.py c2 --batch --modes dense > gpurun_out/r3_dense_c2b.json 2> gpurun_out/r3_dense_c2b.err || exit 1
cat gpurun_out/r3_dense_c2b.json
timeout -k 10 300 python tools/bench_dense.py c5 --width 4096 --modes dense > gpurun_out/r3_dense_c5b.json 2> gpurun_out/r3_dense_c5b.err || exit 1
cat gpurun_out/r3_dense_c5b.json
