#!/usr/bin/env python3
"""HBM traffic per k_pull launch from two rocprofv3 PMC passes of bench.py.

    rocprofv3 --pmc FETCH_SIZE -d <fdir> -o run --output-format csv -- python bench.py ...
    rocprofv3 --pmc WRITE_SIZE -d <wdir> -o run --output-format csv -- python bench.py ...
    python tools/pmc_traffic.py <fdir>/run_counter_collection.csv <wdir>/run_counter_collection.csv \
        --timed K --out profiles/pmc_C3.json

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide
coalesced 16-B-per-lane read, which is the access shape of k_pull's neighbour-row loads, so
read bytes = 2 x FETCH_SIZE.  WRITE_SIZE reads exactly for 16-B-per-lane stores.  Both are in
KiB.  The average is taken over the last K k_pull dispatches (the bench's timed window).
"""
import argparse
import csv
import json
from collections import defaultdict


def per_dispatch(path, counter, kernel):
    vals = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        d = int(r["Dispatch_Id"])
        vals[d] += float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    ids = sorted(d for d in vals if kernel in names[d])
    return [vals[d] for d in ids]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--timed", type=int, required=True)
    ap.add_argument("--passes", type=int, default=1,
                    help="engine passes in the run (share shards per GPU): the timed "
                         "dispatches are the last K of each pass")
    ap.add_argument("--kernel", default="k_pull<", help="substring of the kernel name")
    ap.add_argument("--bench-json", help="the JSON line the profiled bench.py printed: its config "
                                         "is recorded so bench.py attaches this traffic only to "
                                         "lines of the same configuration")
    ap.add_argument("--out")
    a = ap.parse_args()
    def timed(v):  # the last K dispatches of each engine pass
        P = max(a.passes, 1)
        per = len(v) // P
        return [x for q in range(P) for x in v[q * per:(q + 1) * per][-a.timed:]]

    f = timed(per_dispatch(a.fetch_csv, "FETCH_SIZE", a.kernel))
    w = timed(per_dispatch(a.write_csv, "WRITE_SIZE", a.kernel))
    fetch_kib = sum(f) / max(len(f), 1)
    write_kib = sum(w) / max(len(w), 1)
    out = {
        "kernel": a.kernel,
        "launches": [len(f), len(w)],
        "fetch_size_kib_avg": fetch_kib,
        "write_size_kib_avg": write_kib,
        "read_bytes_per_launch": 2 * fetch_kib * 1024,
        "write_bytes_per_launch": write_kib * 1024,
        "hbm_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024,
        "note": "read = 2 x FETCH_SIZE (gfx950 half-count for 16-B/lane reads), KiB -> bytes",
    }
    if a.bench_json:
        with open(a.bench_json) as fh:
            line = json.loads([ln for ln in fh.read().splitlines() if ln.startswith("{")][-1])
        out["config"] = {"workload": "C4" if "10M nodes" in line["config"]["workload"] else "C3",
                         "warmup": line["warmup"], "steps": line["steps"],
                         "live_words_per_node": line["config"]["live_words_per_node"],
                         "pull_variant": line["roofline"]["pull_variant"]}
        roof = line["roofline"]
        kern = roof.get("kernels") or {}
        src = kern.get("k_pull_young" if "young" in a.kernel else "k_pull") or roof
        out["algorithmic_bytes_per_launch"] = src["bytes_per_launch"]
        out["traffic_over_algorithmic"] = out["hbm_bytes_per_launch"] / src["bytes_per_launch"]
    s = json.dumps(out, indent=1)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
