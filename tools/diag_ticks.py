#!/usr/bin/env python3
"""Diagnostic: per-tick pull counters of one share shard of the C4 bench (bench.py's setup).

    python tools/diag_ticks.py [--shards 8] [--rule tick|hash] [--ticks 16] [--warmup 5]

Ramps shard --shard of S exactly as bench.py does (its shard rule and fresh-tile flag), then runs the ticks one at a time, resetting the
device tallies before each (Engine.reset_timing), and prints one JSON line per tick: the pull
phase and kernel times, k_pull's items / gathering items / peer-row loads / occupancy reads /
own-seen reads, and k_pull_young's slot lines -- the per-age costs of DESIGN.md §5."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "p2p-gossip-simulation-ns3_amd"))
import gossip  # noqa: E402
import gossip.workloads as WL  # noqa: E402
from bench import L_NS, SLICE_NS, T0_NS, T_CUT_NS, shard_flags  # noqa: E402

FIELDS = ("pull_ms", "young_ms", "pull_phase_ms", "pull_launches", "young_launches", "pull_items",
          "pull_gather_items", "pull_pair_edges", "pull_col_ids", "pull_nz_reads", "pull_seen_reads",
          "pull_sat_skips", "pull_bytes_moved", "young_slot_lines", "young_bytes_moved",
          "young_skip_ticks", "pull_push_tiles", "pull_pushw_tiles", "pull_marks", "young_list_lines",
          "young_rows_written", "young_fresh_lines", "young_fallback_rows")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--rule", choices=["tick", "hash"], default="tick")
    ap.add_argument("--ticks", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--fresh-tiles", choices=["auto", "on", "off"], default="auto")
    ap.add_argument("--option", action="append", default=[], help="engine option name=value (repeatable)")
    a = ap.parse_args()
    n = WL.CONFIGS["C4"]["nodes"]
    topo = WL.topology("C4", nodes=n, threads=a.threads)
    ev, _ = WL.slice_schedule(n, WL.CONFIGS["C4"]["node_seed"], SLICE_NS,
                              SLICE_NS + (a.warmup + a.ticks + 1) * L_NS, threads=a.threads)
    flags = gossip.F_TIMING | shard_flags(a.rule, a.fresh_tiles)
    eng = gossip.Engine(n, L_NS, T0_NS, T_CUT_NS, flags=flags, shard_rank=a.shard, shard_count=a.shards)
    try:
        for o in a.option:
            k, v = o.split("=")
            eng.set_option(k, int(v))
        eng.set_topology(topo)
        eng.set_schedule(ev)
        t = SLICE_NS // L_NS + a.warmup
        eng.run(t)
        eng.sync()
        for _ in range(a.ticks):
            e0 = eng.counters().edge_events
            eng.reset_timing()
            t += 1
            eng.run(t)
            eng.sync()
            c = eng.counters()
            row = {"tick": t, "edge_events": c.edge_events - e0}
            row.update({f: getattr(c, f) for f in FIELDS})
            print(json.dumps(row), flush=True)
    finally:
        eng.close()


if __name__ == "__main__":
    main()
