#!/usr/bin/env python3
"""Per-tick diagnostics of the engine on the C3 workload (GPU): window width, pull time,
bytes moved, pair-edge reads, edge events.  Syncs after every tick (diagnostic only).

    python tools/diag_ticks.py [--ticks 80] [--nodes 1000000]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-gossip-simulation-ns3_amd"))
import gossip  # noqa: E402

T0, L, TCUT = 5_000_000_000, 5_000_000, 59_900_000_000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ticks", type=int, default=80)
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--deg", type=float, default=16.0)
    ap.add_argument("--max-words", type=int, default=0)
    a = ap.parse_args()
    n = a.nodes
    topo = gossip.Topology.gnp(n, a.deg / (n - 1), 3, gossip.TOPO_SKIP, threads=16)
    ev = gossip.make_schedule(n, 1000, T0, TCUT, t_gen_end_ns=T0 + (a.ticks + 1) * L, threads=16)
    eng = gossip.Engine(n, L, T0, TCUT, flags=gossip.F_TIMING, max_words=a.max_words)
    eng.set_topology(topo)
    eng.set_schedule(ev)
    t0 = eng.first_tick
    prev = eng.counters()
    print("tick words pull_ms moved_GB pair_edges_M edge_events_G births", flush=True)
    for k in range(a.ticks):
        eng.run(t0 + k + 1)
        eng.sync()
        c = eng.counters()
        births = int(((ev["ns"] // L) == t0 + k).sum())
        print(f"{t0 + k} {c.words_hw} {c.pull_ms - prev.pull_ms:.3f} "
              f"{(c.pull_bytes_moved - prev.pull_bytes_moved) / 1e9:.2f} "
              f"{(c.pull_pair_edges - prev.pull_pair_edges) / 1e6:.1f} "
              f"{(c.edge_events - prev.edge_events) / 1e9:.2f} {births}", flush=True)
        prev = c


if __name__ == "__main__":
    main()
