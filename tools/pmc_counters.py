#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per dispatch of one kernel over its last K dispatches.

    python tools/pmc_counters.py --timed K [--kernel k_pull] <dir>/run_counter_collection.csv ...
"""
import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csvs", nargs="+")
    ap.add_argument("--timed", type=int, required=True)
    ap.add_argument("--kernel", default="k_pull")
    a = ap.parse_args()
    out = {}
    for path in a.csvs:
        vals = defaultdict(lambda: defaultdict(float))
        names = {}
        for r in csv.DictReader(open(path)):
            d = int(r["Dispatch_Id"])
            vals[r["Counter_Name"]][d] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
        for c, per in vals.items():
            ids = sorted(d for d in per if a.kernel in names[d])[-a.timed:]
            if ids:
                out[c] = sum(per[d] for d in ids) / len(ids)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
