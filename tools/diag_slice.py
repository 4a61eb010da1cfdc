#!/usr/bin/env python3
"""Diagnostic: the bench's warm-start slice vs the continuous run (tests/test_c3_gpu.py).

    python tools/diag_slice.py [--nodes N] [--variants]

Prints, per engine variant, how many nodes' counter deltas over the timed ticks differ between
the continuous run (every generation from t = 5 s) and the slice replay, and the signed sum of
the differences."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-gossip-simulation-ns3_amd"))
import gossip  # noqa: E402
import gossip.workloads as W  # noqa: E402


def deltas(topo, ev, t0, t1, opts):
    eng = gossip.Engine(topo.num_nodes, W.L_NS, W.T0_NS, W.T_CUT_NS)
    for k, v in opts:
        eng.set_option(k, v)
    eng.set_topology(topo)
    eng.set_schedule(ev)
    eng.run(t0)
    eng.sync()
    a = eng.stats()
    eng.run(t1)
    eng.sync()
    b = eng.stats()
    c = eng.counters()
    eng.close()
    return {k: getattr(b, k).astype(np.int64) - getattr(a, k).astype(np.int64) for k in ("gen", "recv", "sent", "processed")}, c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--variants", action="store_true")
    ap.add_argument("--life", type=int, default=W.LIFE_TICKS)
    a = ap.parse_args()
    topo = W.topology("C3", nodes=a.nodes)
    n = topo.num_nodes
    seed = W.CONFIGS["C3"]["node_seed"]
    t0 = W.SLICE_NS // W.L_NS + 5
    t1 = t0 + 20
    ev = gossip.make_schedule(n, seed, W.T0_NS, W.T_CUT_NS, t_gen_end_ns=t1 * W.L_NS, threads=16)
    sl, info = W.slice_schedule(n, seed, W.SLICE_NS, t1 * W.L_NS, life_ticks=a.life)
    variants = [("default", ())]
    if a.variants:
        variants += [("late_age 0", (("late_age", 0),)), ("pull_gate 0", (("pull_gate", 0),)),
                     ("late 0 + gate 0", (("late_age", 0), ("pull_gate", 0)))]
    ref = None
    for name, opts in variants:
        dc, cc = deltas(topo, ev, t0, t1, opts)
        ds, cs = deltas(topo, sl, t0, t1, opts)
        if ref is None:
            ref = dc
        out = {"nodes": n, "variant": name, "life": a.life, "slice_info": info,
               "words_hw": [cc.words_hw, cs.words_hw], "cap": [cc.words_cap, cs.words_cap]}
        for k in dc:
            diff = dc[k] - ds[k]
            out[k] = {"nodes_differ": int(np.count_nonzero(diff)), "sum_cont_minus_slice": int(diff.sum()),
                      "cont_vs_default_cont": int(np.count_nonzero(dc[k] - ref[k]))}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
