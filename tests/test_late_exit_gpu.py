"""Late-tile bottom-up early exit in k_pull (option late_age, WF_LATE; on for every tile of a CSR
pull by default) against ORACLE A.

For a tile at least `late_age` ticks old, k_pull stops reading a node's peer rows at the first
batch whose OR covers every bit the node can still take (live last tick, unseen, kept): the
remaining rows cannot change `new` (p2pnode.cc:189 -- a share already in processedShares is
dropped), so the counters and the first-contact trace must stay bit-exact, with id groups,
a cut inside a tick and young tiles on or off, while fewer peer rows are read.
"""
import numpy as np
import pytest

from cases import T0

pytestmark = pytest.mark.gpu

STATS = ("gen", "recv", "fwd", "sent", "processed", "peers", "sockets")


def _engine(gossip, topo, ev, lat, t_cut, opts, flags):
    eng = gossip.Engine(topo.num_nodes, lat, T0, t_cut, flags=flags)
    for k, v in opts.items():
        eng.set_option(k, v)
    eng.set_topology(topo)
    eng.set_schedule(ev)
    eng.run()
    eng.sync()
    return eng


@pytest.fixture(scope="module")
def late_case(gossip, oracle):
    # one workload and ONE ORACLE A run (the costly part) for every variant below
    n = 6000
    topo = gossip.Topology.gnp(n, 16.0 / (n - 1), 91, gossip.TOPO_SKIP)
    lat = gossip.milliseconds_to_ns(5.0)
    t_cut = gossip.seconds_to_ns(6.37)  # a cut inside a tick: keep masks on late words
    ev = gossip.make_schedule(n, 92, T0, t_cut, id_mask=0x3FFF)  # id groups
    a, b = topo.links()
    r = oracle.run_replay(n, lat, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"], trace=True)
    return topo, lat, t_cut, ev, r


@pytest.mark.parametrize("late_age,young", [(1, 0), (3, 0), (4, 1), (2, 1)])
def test_late_exit_matches_oracle(gossip, late_case, late_age, young):
    topo, lat, t_cut, ev, r = late_case
    # a fresh tile per tick keeps the window wider than 64 words: the one-peer-walk-per-node
    # pull (k_pull<32, 1>) that carries the exit
    # (young tiles only up to age 2, so that k_pull still sees tiles with unseen bits)
    yo = dict(young=young, young_age=2) if young else dict(young=0)
    eng = _engine(gossip, topo, ev, lat, t_cut, dict(yo, late_age=late_age),
                  gossip.F_TRACE | gossip.F_TILE_PER_TICK)
    st = eng.stats()
    base = _engine(gossip, topo, ev, lat, t_cut, dict(yo, late_age=0), gossip.F_TILE_PER_TICK)
    assert eng.counters().pull_pair_edges < base.counters().pull_pair_edges  # the exit was taken
    base.close()
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(r, k)), (late_age, k)
    node, sid, tick, hop, via = eng.trace()
    tn, ti, tt, th, tv = r.trace
    ek, ok = np.lexsort((sid, node)), np.lexsort((ti, tn))
    assert np.array_equal(node[ek], tn[ok]) and np.array_equal(sid[ek], ti[ok])
    assert np.array_equal(tick[ek], tt[ok] // lat) and np.array_equal(hop[ek], th[ok])
    assert np.array_equal(via[ek], tv[ok])  # ReceiveShare vs own generation (p2pnode.cc:115-120,155-165)
    eng.close()


def test_late_exit_reads_fewer_rows(gossip):
    # 200k nodes, degree 16: late tiles (dense frontier, few unseen bits) stop after one batch
    n = 200_000
    topo = gossip.Topology.gnp(n, 16.0 / (n - 1), 93, gossip.TOPO_SKIP, threads=16)
    lat = gossip.milliseconds_to_ns(5.0)
    t_cut = gossip.seconds_to_ns(5.4)
    ev = gossip.make_schedule(n, 94, T0, t_cut)
    runs = {}
    for late in (0, 4):
        eng = _engine(gossip, topo, ev, lat, t_cut, dict(late_age=late, young=0), gossip.F_TILE_PER_TICK)
        runs[late] = (eng.stats(), eng.counters())
        eng.close()
    for k in STATS:
        assert np.array_equal(getattr(runs[0][0], k), getattr(runs[4][0], k)), k
    assert runs[4][1].pull_pair_edges < runs[0][1].pull_pair_edges


@pytest.mark.parametrize("gate", [1, 0])
def test_seen_gate_with_wide_peer_lists(gossip, oracle, gate):
    # k_pull<32, 1> (windows wider than 64 words) serves a node with one 32-lane group; nodes
    # with more peers than that must never be gated on the first group's occupancy alone (the
    # occupancy gate of the own-seen loads, option pull_gate; a C3 run lost receptions at
    # 37-peer nodes when the one-group test read the row pointers of inactive lanes).  Average
    # degree 40: most nodes have > 32 peers.
    n = 3000
    topo = gossip.Topology.gnp(n, 40.0 / (n - 1), 95, gossip.TOPO_EXACT)
    lat = gossip.milliseconds_to_ns(5.0)
    t_cut = gossip.seconds_to_ns(5.6)
    ev = gossip.make_schedule(n, 96, T0, t_cut)
    eng = _engine(gossip, topo, ev, lat, t_cut, dict(pull_gate=gate, young=0), gossip.F_TILE_PER_TICK)
    st = eng.stats()
    assert eng.counters().words_hw > 64  # the one-group-per-node pull
    eng.close()
    a, b = topo.links()
    r = oracle.run_replay(n, lat, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"])
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(r, k)), (gate, k)
