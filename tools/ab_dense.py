#!/usr/bin/env python3
"""One short line from a tools/bench_dense.py output: python tools/ab_dense.py <name> <file>."""
import json
import sys

d = json.loads([ln for ln in open(sys.argv[2]).read().splitlines() if ln.startswith("{")][-1])
print(sys.argv[1], d["workload"][:3], "phase_ms_avg %.4f" % d["phase_ms_avg"], "util_phase %.3f" % d["mfma_util_phase"],
      "pull_ms_avg %.4f" % d["pull_ms_avg"], "ops %.4g" % d["dense_ops"], "same", d["identical_to_first"])
