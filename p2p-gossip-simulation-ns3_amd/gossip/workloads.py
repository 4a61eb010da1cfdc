"""The BASELINE.json configurations as inputs of the engine (host side; shared by bench.py,
tools/ and the GPU tests so that the benchmarked and the tested workloads are the same).

  C2  dense  G(n,p) 4,096 nodes, p = 0.3, 60 s, real schedule
  C3  sparse G(n,p) 1M nodes, average degree 16
  C4  sparse G(n,p) 10M nodes, average degree 16 (the headline metric's configuration)
  C5  dense  G(n,p) 65,536 nodes, p = 0.3, 4,096 concurrent shares at Philox-chosen origins

A C3/C4 "slice" is a window of steady-state ticks of the reference's continuous run.  Its
schedule is every generation of the window plus the LIFE ticks before it (the floods still
alive when the window opens: ~eccentricity ticks) plus every earlier generation of an id that
occurs there -- so an id generated twice (GenerateUniqueShareId collides above 128,849 nodes,
p2pnode.cc:201-209) meets the seen-sets (p2pnode.cc:189) its earlier flood left, as in the
continuous run.
"""
from __future__ import annotations

import numpy as np

from . import (GEN_EVENT_DTYPE, TOPO_EXACT, TOPO_SKIP, Topology, events_from_arrays,
               make_schedule)

T0_NS = 5_000_000_000          # makeconnections, Seconds(5) (p2pnetwork.cc:93)
L_NS = 5_000_000               # --Latency 5 ms
T_CUT_NS = 59_900_000_000      # PrintStatistics at simTime - 0.1 (p2pnetwork.cc:206)
SLICE_NS = 10_000_000_000      # steady-state slice start (tick 2000): the U(2,5) s renewal
                               # density has settled at 1/3.5 s per node by then
LIFE_TICKS = 16                # > the flood lifetime of C3/C4 (eccentricity ~8-9)

CONFIGS = {
    "C2": dict(nodes=4096, p=0.3, topo_seed=2, node_seed=2000, kind=TOPO_EXACT),
    "C3": dict(nodes=1_000_000, avg_degree=16, topo_seed=3, node_seed=1000, kind=TOPO_SKIP),
    "C4": dict(nodes=10_000_000, avg_degree=16, topo_seed=4, node_seed=2000, kind=TOPO_SKIP),
    "C5": dict(nodes=65536, p=0.3, topo_seed=5, width=4096, origin_seed=12345, kind=TOPO_SKIP),
}


def edge_prob(cfg: dict, nodes: int | None = None) -> float:
    n = nodes or cfg["nodes"]
    return cfg["p"] if "p" in cfg else cfg["avg_degree"] / (n - 1)


def topology(name: str, nodes: int | None = None, threads: int = 16) -> Topology:
    cfg = CONFIGS[name]
    n = nodes or cfg["nodes"]
    return Topology.gnp(n, edge_prob(cfg, n), cfg["topo_seed"], cfg["kind"], threads=threads)


def slice_schedule(n: int, node_seed: int, t_slice_ns: int, t_end_ns: int,
                   life_ticks: int = LIFE_TICKS, threads: int = 16):
    """Generations of the slice [t_slice - life_ticks*L, t_end) of the reference's run, plus all
    earlier generations (>= 5 s) of the ids that occur in it.  Returns (events, info)."""
    ev = make_schedule(n, node_seed, T0_NS, T_CUT_NS, t_gen_end_ns=t_end_ns, threads=threads)
    t_lo = t_slice_ns - life_ticks * L_NS
    win = ev["ns"] >= t_lo
    early = ~win & np.isin(ev["share_id"], np.unique(ev["share_id"][win]))
    out = ev[win | early]  # still sorted by (ns, node)
    info = dict(t_lo_ns=int(t_lo), window_generations=int(win.sum()),
                earlier_same_id=int(early.sum()), life_ticks=life_ticks)
    return np.ascontiguousarray(out, GEN_EVENT_DTYPE), info


def c5_flood(n: int | None = None, width: int | None = None):
    """C5's flood batch: `width` concurrent shares, distinct ids, at Philox-chosen origins, all
    generated 1 us into the first tick after t_start."""
    cfg = CONFIGS["C5"]
    n = n or cfg["nodes"]
    width = width or cfg["width"]
    rng = np.random.Generator(np.random.Philox(cfg["origin_seed"]))
    origins = rng.choice(n, size=width, replace=False)
    return events_from_arrays(np.full(width, T0_NS + 1000, np.int64), origins,
                              np.arange(1, width + 1, dtype=np.uint32))
