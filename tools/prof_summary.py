#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run of bench.py for profiles/.

    python tools/prof_summary.py <prof_dir> <run_name> --timed K [--out profiles/x.json]

Reports every kernel's call count / average duration (from <run>_kernel_stats.csv) and the
average duration of the LAST K k_pull dispatches (the bench's timed window), which is the
number bench.py's live HIP-event average must agree with.
"""
import argparse
import csv
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("run")
    ap.add_argument("--timed", type=int, required=True)
    ap.add_argument("--passes", type=int, default=1,
                    help="engine passes in the run (share shards per GPU): the timed "
                         "dispatches are the last K of each pass")
    ap.add_argument("--kernel", default="k_pull<", help="substring of the kernel name")
    ap.add_argument("--phase-with", help="substring of a second kernel launched beside --kernel "
                                          "every tick (on another stream): also report the "
                                          "timed ticks' phase = first start to last end of both")
    ap.add_argument("--out")
    a = ap.parse_args()
    stats = list(csv.DictReader(open(os.path.join(a.prof_dir, f"{a.run}_kernel_stats.csv"))))
    trace = list(csv.DictReader(open(os.path.join(a.prof_dir, f"{a.run}_kernel_trace.csv"))))
    pulls = [r for r in trace if a.kernel in r["Kernel_Name"]]
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in pulls]
    P = max(a.passes, 1)
    per = len(dur) // P
    timed = [x for q in range(P) for x in dur[q * per:(q + 1) * per][-a.timed:]]
    out = {
        "kernels": [{"name": r["Name"], "calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                     "total_ms": float(r["TotalDurationNs"]) / 1e6, "pct": float(r["Percentage"])}
                    for r in stats],
        "timed_kernel": a.kernel,
        "timed_launches": len(timed),
        "timed_avg_ms": sum(timed) / max(len(timed), 1),
        "timed_min_ms": min(timed) if timed else None,
        "timed_max_ms": max(timed) if timed else None,
        "vgpr": int(pulls[-1]["VGPR_Count"]) if pulls else None,
        "sgpr": int(pulls[-1]["SGPR_Count"]) if pulls else None,
        "lds_bytes": int(pulls[-1]["LDS_Block_Size"]) if pulls else None,
        "grid": int(pulls[-1]["Grid_Size_X"]) if pulls else None,
    }
    if a.phase_with:
        other = [r for r in trace if a.phase_with in r["Kernel_Name"]]
        x = [r for q in range(P) for r in pulls[q * per:(q + 1) * per][-a.timed:]]
        # the partner of a timed dispatch: the other kernel's dispatch that started closest to it
        y = [min(other, key=lambda o: abs(int(o["Start_Timestamp"]) - int(p["Start_Timestamp"]))) for p in x]
        ph = [(max(int(p["End_Timestamp"]), int(o["End_Timestamp"])) -
               min(int(p["Start_Timestamp"]), int(o["Start_Timestamp"]))) / 1e6 for p, o in zip(x, y)]
        yd = [(int(o["End_Timestamp"]) - int(o["Start_Timestamp"])) / 1e6 for o in y]
        out["phase_with"] = a.phase_with
        out["phase_ticks"] = len(ph)
        out["phase_avg_ms"] = sum(ph) / max(len(ph), 1)
        out["phase_with_avg_ms"] = sum(yd) / max(len(yd), 1)
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
