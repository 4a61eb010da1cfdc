#!/usr/bin/env python3
"""DENSE phase utilisation from a rocprofv3 kernel trace of tools/bench_dense.py.

    python tools/dense_trace.py <trace_dir>/run_kernel_trace.csv <bench_dense line (json file)> [--out f.json]

Only the line's own run counts: its last `pull_launches` dispatches (tools/bench_dense.py runs the
workload once untimed first).  Per tick the DENSE phase is the span from the first start to the last end of its kernels --
k_dense_fused (round 5), or k_transpose + k_dense_bits + k_dense_dedup (the three-kernel path) --
in the order they were dispatched (the stamp kernels k_phase_start / k_phase_acc, k_births and
copies are not part of it).  int8 MFMA utilisation = the line's dense_ops (2 x M x N x K of the
stages computed) / summed spans / 5 POPS (MI355X_MICROARCH.md: 2x the 2.5 PF dense bf16 rate).
"""
import argparse
import csv
import json

PHASE = ("k_transpose", "k_dense_bits", "k_dense_dedup", "k_dense_fused")
INT8_PEAK_OPS = 5.0e15


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("line")
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    rows.sort()
    spans, kerns, cur, ck = [], [], None, {}
    for s, e, k in rows:
        if k in PHASE:
            if cur is None:
                cur, ck = [s, e], {}
            else:
                cur[1] = max(cur[1], e)
            ck[k] = ck.get(k, 0.0) + (e - s) / 1e3
        elif cur is not None:  # the first non-phase kernel after the phase closes it
            spans.append((cur[1] - cur[0]) / 1e3)
            kerns.append(ck)
            cur = None
    if cur is not None:
        spans.append((cur[1] - cur[0]) / 1e3)
        kerns.append(ck)
    line = json.loads([ln for ln in open(a.line).read().splitlines() if ln.startswith("{")][-1])
    ops = line["dense_ops"]
    spans = spans[-line["pull_launches"]:]  # (the measured run; a warm-up run precedes it)
    kern = {}
    for ck in kerns[-line["pull_launches"]:]:
        for k, v in ck.items():
            kern[k] = kern.get(k, 0.0) + v
    tot = sum(spans)
    ksum = sum(kern.values())
    out = {
        "source": a.trace,
        "workload": line["workload"],
        "dispatches": len(spans),
        "span_us_total": tot,
        "span_us_mean": tot / max(len(spans), 1),
        "kernel_us_total": kern,
        "dense_ops": ops,
        "mfma_util_phase_by_trace_span": ops / (tot * 1e-6) / INT8_PEAK_OPS if tot else None,
        "mfma_util_phase_kernels_only": ops / (ksum * 1e-6) / INT8_PEAK_OPS if ksum else None,
        "spans_us": [round(x, 1) for x in spans],
    }
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
