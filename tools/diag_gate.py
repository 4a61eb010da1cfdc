#!/usr/bin/env python3
"""Diagnostic: k_pull's occupancy gate of the own-seen loads (option pull_gate) on C3's continuous
run.  Steps an engine with the gate and one without, tick by tick, and reports the first tick at
which their per-node receive counters differ (and the nodes); optionally with every share id made
unique (no id groups)."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-gossip-simulation-ns3_amd"))
import gossip  # noqa: E402
import gossip.workloads as W  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--unique", action="store_true")
    ap.add_argument("--ticks", type=int, default=1025)
    ap.add_argument("--opt", action="append", default=[], help="extra option k=v for both engines")
    a = ap.parse_args()
    topo = W.topology("C3", nodes=a.nodes)
    n = topo.num_nodes
    t_end = W.T0_NS // W.L_NS + a.ticks
    ev = gossip.make_schedule(n, W.CONFIGS["C3"]["node_seed"], W.T0_NS, W.T_CUT_NS, t_gen_end_ns=t_end * W.L_NS,
                              threads=16)
    if a.unique:
        ev["share_id"] = np.arange(1, len(ev) + 1, dtype=np.uint32)
    engs = []
    for gate in (0, 1):
        e = gossip.Engine(n, W.L_NS, W.T0_NS, W.T_CUT_NS)
        e.set_option("pull_gate", gate)
        for kv in a.opt:
            k, v = kv.split("=")
            e.set_option(k, int(v))
        e.set_topology(topo)
        e.set_schedule(ev)
        engs.append(e)
    rp, col, _ = topo.csr()
    t = engs[0].first_tick
    first = None
    while t < t_end:
        t += 1
        for e in engs:
            e.run(t)
        s0, s1 = engs[0].stats(), engs[1].stats()
        d = np.flatnonzero(s0.recv != s1.recv)
        if len(d):
            v = int(d[0])
            first = {"tick": t, "nodes_differ": len(d), "nodes": d[:20].tolist(),
                     "recv_gate0": s0.recv[d[:20]].tolist(), "recv_gate1": s1.recv[d[:20]].tolist(),
                     "deg_first": int(rp[v + 1] - rp[v]), "peers_first": col[rp[v]:rp[v + 1]].tolist(),
                     "words_hw": engs[0].counters().words_hw}
            break
    print(json.dumps({"nodes": n, "unique_ids": a.unique, "opts": a.opt, "ticks_run": t - engs[0].first_tick,
                      "first_difference": first}), flush=True)
    for e in engs:
        e.close()


if __name__ == "__main__":
    main()
