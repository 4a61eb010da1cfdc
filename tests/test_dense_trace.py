"""tools/dense_trace.py: the DENSE phase utilisation from a rocprofv3 kernel trace (CPU only).

A phase is the span from the first start to the last end of the phase's kernels of one dispatch,
closed by the first other kernel; only the line's own run counts (its last `pull_launches`
dispatches: tools/bench_dense.py runs an untimed warm-up first).
"""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "dense_trace.py")


def _write_trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        for name, s, e in rows:
            w.writerow({"Kernel_Name": name, "Start_Timestamp": s, "End_Timestamp": e})


def test_spans_of_the_measured_run_only(tmp_path):
    fused = "(anonymous namespace)::k_dense_fused((anonymous namespace)::FusedArgs)"  # (rocprofv3 names)
    tr = "(anonymous namespace)::k_transpose(unsigned long*)"
    births = "(anonymous namespace)::k_births((anonymous namespace)::BirthArgs)"
    rows = [
        # warm-up run: one dispatch with a long first-launch gap (excluded)
        (tr, 0, 5_000), (fused, 140_000, 150_000), (births, 160_000, 170_000),
        # measured run: two dispatches, the first with k_transpose
        (tr, 1_000_000, 1_004_000), (fused, 1_006_000, 1_106_000), (births, 1_110_000, 1_120_000),
        (fused, 1_200_000, 1_300_000), (births, 1_310_000, 1_320_000),
    ]
    trace = tmp_path / "run_kernel_trace.csv"
    _write_trace(trace, rows)
    ops = 5.0e15 * 206e-6 * 0.5  # half the int8 peak over the two measured spans (106 + 100 us)
    line = tmp_path / "line.json"
    line.write_text(json.dumps({"workload": "test", "dense_ops": ops, "pull_launches": 2}) + "\n")
    out = subprocess.run([sys.executable, TOOL, str(trace), str(line)], capture_output=True, text=True, check=True)
    d = json.loads(out.stdout)
    assert d["dispatches"] == 2
    assert d["spans_us"] == [106.0, 100.0]
    assert abs(d["mfma_util_phase_by_trace_span"] - 0.5) < 1e-9
    assert d["kernel_us_total"] == {"k_transpose": 4.0, "k_dense_fused": 200.0}
