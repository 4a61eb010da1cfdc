"""NS-3 handshake window.

makeconnections (p2pnetwork.cc:99-150) runs at t_start: for a key (a,b), a adds b to peers and
connects; a's TCP socket is ESTABLISHED about two hops later, and every share a sends before
that is buffered behind "REGISTER:a", which HandleRead parses as a registration only
(p2pnode.cc:178-188): counted as sent, lost.  REGISTER reaches b about three hops after
t_start and only then appends a to peers(b).  Model: est = 2L, reg = 3L, REGISTER before any
other event of its nanosecond.  ORACLE A (CPU) against hand-derived counts; the HIP engine
(GOSSIP_F_HANDSHAKE) against ORACLE A bit for bit, first-contact traces included.
"""
import numpy as np
import pytest

from cases import BIG, L, T0

STATS = ("gen", "recv", "fwd", "sent", "processed", "peers", "sockets")
HS = (2 * L, 3 * L)

# path 0-1-2 with keys (0,1) and (1,2): node 0 connects to 1, node 1 connects to 2
LINKS = [(0, 1), (1, 2)]
EVENTS = [
    (T0 + 100, 0, 11),        # tick +0: before ESTABLISHED -> counted, sent to 1, lost
    (T0 + L + 5, 2, 12),      # tick +1: node 2 only accepts -> peers empty, not counted
    (T0 + 2 * L + 7, 1, 13),  # tick +2: connector side only: 1 -> 2 delivered at +3L+7,
]                             #          2 (REGISTER from 1 arrived at +3L) echoes it back
EXPECT = dict(gen=[1, 1, 0], recv=[0, 0, 1], fwd=[0, 0, 1], sent=[1, 1, 1],
              processed=[1, 1, 1], peers=[1, 2, 1], sockets=[1, 2, 1])


def _split(links):
    return [a for a, _ in links], [b for _, b in links]


def test_oracle_handshake_hand_case(oracle):
    a, b = _split(LINKS)
    ev = np.array(EVENTS, dtype=np.int64)
    r = oracle.run_replay(3, L, T0, BIG, a, b, ev[:, 0], ev[:, 1], ev[:, 2], handshake=HS)
    for k, want in EXPECT.items():
        assert getattr(r, k).tolist() == want, (k, getattr(r, k))


def test_oracle_handshake_changes_only_the_start(oracle):
    # same topology and schedule: peers/sockets/gens agree; the window only loses early shares
    kw = dict(num_nodes=40, connection_prob=0.1, sim_time_s=12.0, topo_seed=3, node_seed=77)
    ideal = oracle.run_reference(**kw)
    hs = oracle.run_reference(register_delay_ns=HS[1], est_delay_ns=HS[0], **kw)
    for k in ("gen", "peers", "sockets"):
        assert np.array_equal(getattr(ideal, k), getattr(hs, k)), k
    assert np.array_equal(hs.fwd, hs.recv)
    assert int(hs.recv.sum()) <= int(ideal.recv.sum())


@pytest.mark.gpu
def test_engine_handshake_hand_case(gossip):
    a, b = _split(LINKS)
    topo = gossip.Topology.from_links(3, a, b)
    ev = np.array(EVENTS, dtype=np.int64)
    eng = gossip.Engine(3, L, T0, BIG, flags=gossip.F_HANDSHAKE)
    eng.set_topology(topo)
    eng.set_schedule(gossip.events_from_arrays(ev[:, 0], ev[:, 1], ev[:, 2]))
    eng.run()
    eng.sync()
    st = eng.stats()
    for k, want in EXPECT.items():
        assert getattr(st, k).tolist() == want, (k, getattr(st, k))


@pytest.mark.gpu
@pytest.mark.parametrize("n,p,sim,lat,seed", [(10, 0.3, 60.0, 5.0, 1), (254, 0.3, 12.0, 5.0, 4),
                                              (120, 0.02, 12.0, 1.0, 7), (4096, 16 / 4095, 6.0, 5.0, 21)])
def test_engine_handshake_matches_oracle(gossip, oracle, n, p, sim, lat, seed):
    lat_ns = gossip.milliseconds_to_ns(lat)
    s = gossip.P2PGossipNetworkSimulation(n, topo_seed=seed, node_seed=seed + 1000,
                                          topology_kind=gossip.TOPO_EXACT,
                                          flags=gossip.F_HANDSHAKE | gossip.F_TRACE)
    s.CreateRandomTopology(p, lat)
    st = s.Start(sim)
    r = oracle.run_reference(num_nodes=n, connection_prob=p, sim_time_s=sim, latency_ms=lat,
                             topo_seed=seed, node_seed=seed + 1000, register_delay_ns=3 * lat_ns,
                             est_delay_ns=2 * lat_ns, trace=True)
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(r, k)), k
    node, sid, tick, hop, via = s.engine.trace()
    tn, ti, tt, th, tv = r.trace
    ek, ok = np.lexsort((sid, node)), np.lexsort((ti, tn))
    assert np.array_equal(node[ek], tn[ok]) and np.array_equal(sid[ek], ti[ok])
    assert np.array_equal(tick[ek], tt[ok] // lat_ns) and np.array_equal(hop[ek], th[ok])
    assert np.array_equal(via[ek], tv[ok])


@pytest.mark.gpu
def test_engine_handshake_rejects_unaligned_start(gossip):
    with pytest.raises(gossip.GossipError, match="multiple of the latency"):
        gossip.Engine(10, 3_700_000, T0, T0 + 10**9, flags=gossip.F_HANDSHAKE)
