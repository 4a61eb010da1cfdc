"""ORACLE A reproduces the committed golden fixtures (tests/golden/, made by
tests/golden/make_golden.py), and the product's host topology reproduces their link sets."""
import numpy as np
import pytest

import golden_util as G


@pytest.mark.parametrize("name", G.names())
def test_oracle_reproduces_golden(oracle, name):
    g = G.load(name)
    r = oracle.run_reference(**g["params"])
    for k in G.STAT_KEYS:
        assert np.array_equal(getattr(r, k), g[k]), k
    assert np.array_equal(np.array(r.periodic, np.int64).reshape(-1, 4), g["periodic"])
    assert r.edge_events == int(g["edge_events"])


@pytest.mark.parametrize("name", G.names())
def test_product_topology_reproduces_golden_links(gossip, name):
    g = G.load(name)
    p = g["params"]
    t = gossip.Topology.gnp(p["num_nodes"], p["connection_prob"], p["topo_seed"], gossip.TOPO_EXACT)
    a, b = t.links()
    if "link_a" in g:
        assert np.array_equal(a, g["link_a"]) and np.array_equal(b, g["link_b"])
    else:
        assert a.size == int(g["link_count"])
        assert G.links_digest(a, b) == str(g["link_sha256"])
    peers, sockets = t.degrees()
    assert np.array_equal(peers, g["peers"]) and np.array_equal(sockets, g["sockets"])
