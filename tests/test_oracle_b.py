"""ORACLE B (bit-sliced, level-synchronous; distinct ids) agrees with ORACLE A (event-driven)
bit for bit, so it can stand in for A at sizes A's event loop cannot reach (C5: 65,536 nodes,
p = 0.3, ~1.3e9 edge events per share).  CPU only."""
import numpy as np
import pytest

import golden_util as G
from cases import CASES, L, T0

STATS = ("gen", "recv", "fwd", "sent", "processed", "peers", "sockets")


def _both(oracle, n, lat, t_cut, a, b, ev_ns, ev_node, ev_id):
    ra = oracle.run_replay(n, lat, T0, t_cut, a, b, ev_ns, ev_node, ev_id)
    rb = oracle.run_oracle_b(n, lat, t_cut, a, b, ev_ns, ev_node, ev_id, threads=4)
    for k in STATS:
        assert np.array_equal(getattr(ra, k), getattr(rb, k)), k
    assert ra.edge_events == rb.edge_events
    return rb


@pytest.mark.parametrize("c", [c for c in CASES if "collide" not in c["name"]],
                         ids=lambda c: c["name"])
def test_hand_cases(oracle, c):
    a = [x for x, _ in c["links"]]
    b = [y for _, y in c["links"]]
    ev = np.array(c["events"], dtype=np.int64)
    r = _both(oracle, c["n"], L, c["t_cut"], a, b, ev[:, 0], ev[:, 1], ev[:, 2])
    for k, want in c["expect"].items():
        assert getattr(r, k).tolist() == want, k


@pytest.mark.parametrize("name", [x for x in G.names() if "collide" not in x])
def test_goldens(oracle, name):
    g = G.load(name)
    p = g["params"]
    ref = oracle.run_reference(**p)  # the golden's own link keys and generations
    lat = oracle.milliseconds_to_ns(p["latency_ms"])
    t_cut = oracle.seconds_to_ns(p["sim_time_s"] - 0.1)
    gns, gnode, gid = ref.gen_events
    if len(np.unique(gid)) != len(gid):
        pytest.skip("colliding ids: ORACLE B does not apply")
    rb = oracle.run_oracle_b(p["num_nodes"], lat, t_cut, *ref.links, gns, gnode, gid, threads=4)
    for k in STATS:
        assert np.array_equal(getattr(rb, k), g[k]), k
    assert rb.edge_events == int(g["edge_events"])


@pytest.mark.parametrize("n,p,seed,sim_s,lat_ms", [(300, 0.02, 3, 9.0, 2.3), (200, 0.3, 4, 6.0, 5.0),
                                                  (1000, 0.004, 5, 12.0, 7.0)])
def test_random_replays(oracle, gossip, n, p, seed, sim_s, lat_ms):
    topo = gossip.Topology.gnp(n, p, seed, gossip.TOPO_EXACT)
    lat = gossip.milliseconds_to_ns(lat_ms)
    t_cut = gossip.seconds_to_ns(sim_s - 0.1)
    ev = gossip.make_schedule(n, seed + 100, T0, t_cut)
    a, b = topo.links()
    _both(oracle, n, lat, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"])


def test_rejects_colliding_ids(oracle):
    with pytest.raises(RuntimeError, match="distinct"):
        oracle.run_oracle_b(3, L, T0 + 10 * L, [0, 1], [1, 2], [T0, T0 + 1], [0, 2], [5, 5])
