# Round 3: where does the own-seen occupancy gate (pull_gate) change C3's results?
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python tools/diag_gate.py > gpurun_out/r3_gate.json 2> gpurun_out/r3_gate.err || { tail -5 gpurun_out/r3_gate.err; exit 1; }
cat gpurun_out/r3_gate.json
timeout -k 10 400 python tools/diag_gate.py --unique > gpurun_out/r3_gate_u.json 2>> gpurun_out/r3_gate.err || { tail -5 gpurun_out/r3_gate.err; exit 1; }
cat gpurun_out/r3_gate_u.json
timeout -k 10 400 python tools/diag_gate.py --opt late_age=0 --opt pull_lpw=64 > gpurun_out/r3_gate_l64.json 2>> gpurun_out/r3_gate.err || { tail -5 gpurun_out/r3_gate.err; exit 1; }
cat gpurun_out/r3_gate_l64.json
