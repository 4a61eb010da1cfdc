"""Hop-batched runs (GOSSIP_F_HOP_BATCH): generation g of every node is simulated
in batched tick g and the PrintStatistics cut / periodic snapshots are applied per share from
the real generation times.  With unique share ids the floods are independent, so every counter
must equal the tick-by-tick run and ORACLE A bit for bit."""
import numpy as np
import pytest

import golden_util as G
from cases import L, T0

pytestmark = pytest.mark.gpu

STATS = ("gen", "recv", "fwd", "sent", "processed", "peers", "sockets")


@pytest.mark.parametrize("name", [n for n in G.names() if not G.load(n)["params"].get("id_mask")])
def test_hop_batch_golden(gossip, name):
    g = G.load(name)
    p = g["params"]
    sim = gossip.P2PGossipNetworkSimulation(p["num_nodes"], topo_seed=p["topo_seed"],
                                            node_seed=p["node_seed"], topology_kind=gossip.TOPO_EXACT,
                                            flags=gossip.F_HOP_BATCH)
    sim.CreateRandomTopology(p["connection_prob"], p["latency_ms"])
    st = sim.Start(p["sim_time_s"])
    for k in STATS:
        assert np.array_equal(getattr(st, k), g[k]), k
    per = [(gossip.seconds_to_ns(t), gg, pp, s) for t, gg, pp, s in sim.periodic]
    assert np.array_equal(np.array(per, np.int64).reshape(-1, 4), g["periodic"])
    # far fewer steps than ticks of simulated time
    assert sim.engine.counters().ticks < 200


@pytest.mark.parametrize("mode", ["csr", "dense"])
def test_hop_batch_trace_matches_oracle(gossip, oracle, mode):
    n = 512
    topo = gossip.Topology.gnp(n, 0.3, 22, gossip.TOPO_EXACT)
    t_cut = gossip.seconds_to_ns(7.9)
    ev = gossip.make_schedule(n, 23, T0, t_cut)
    m = gossip.MODE_DENSE if mode == "dense" else gossip.MODE_CSR
    eng = gossip.Engine(n, L, T0, t_cut, mode=m, flags=gossip.F_HOP_BATCH | gossip.F_TRACE)
    eng.set_topology(topo)
    eng.set_schedule(ev)
    eng.run()
    eng.sync()
    st = eng.stats()
    a, b = topo.links()
    r = oracle.run_replay(n, L, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"], trace=True)
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(r, k)), k
    node, sid, tick, hop, via = eng.trace()
    tn, ti, tt, th, tv = r.trace
    ek, ok = np.lexsort((sid, node)), np.lexsort((ti, tn))
    assert np.array_equal(node[ek], tn[ok]) and np.array_equal(sid[ek], ti[ok])
    assert np.array_equal(tick[ek], tt[ok] // L) and np.array_equal(hop[ek], th[ok])
    assert np.array_equal(via[ek], tv[ok])


def test_hop_batch_c2_equals_tick_run(gossip):
    # C2: 4,096 nodes, p = 0.3, the full 60 s, periodic stats, on the MFMA path
    n = 4096
    topo = gossip.Topology.gnp(n, 0.3, 2, gossip.TOPO_EXACT)
    t_cut = gossip.seconds_to_ns(59.9)
    ev = gossip.make_schedule(n, 2000, T0, t_cut)
    out = []
    for flags in (0, gossip.F_HOP_BATCH):
        eng = gossip.Engine(n, L, T0, t_cut, mode=gossip.MODE_DENSE, flags=flags)
        eng.set_topology(topo)
        for t in range(10, 60, 10):
            eng.add_snapshot(gossip.seconds_to_ns(t))
        eng.set_schedule(ev)
        eng.run()
        eng.sync()
        out.append((eng.stats(), [eng.snapshot(k) for k in range(5)], eng.counters().ticks))
        eng.close()
    (a, sa, ta), (b, sb, tb) = out
    for k in STATS:
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    assert sa == sb
    assert tb * 100 < ta


def test_hop_batch_rejects_colliding_ids(gossip):
    n = 300
    topo = gossip.Topology.gnp(n, 0.05, 5, gossip.TOPO_EXACT)
    t_cut = gossip.seconds_to_ns(20.0)
    ev = gossip.make_schedule(n, 9, T0, t_cut, id_mask=0xFF)
    eng = gossip.Engine(n, L, T0, t_cut, flags=gossip.F_HOP_BATCH)
    eng.set_topology(topo)
    with pytest.raises(gossip.GossipError, match="unique share ids"):
        eng.set_schedule(ev)
