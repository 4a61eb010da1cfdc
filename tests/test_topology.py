"""Topology builder (product host code) vs the oracle and the reference's fix-up rules.

Reference: CreateRandomTopology p2pnetwork.cc:62-96, ConnectNodes :110-130, makeconnections /
ConnectPeerSockets :99-150, AddPeer p2pnode.cc:77-83, REGISTER branch p2pnode.cc:178-188.
"""
import numpy as np
import pytest

import refrng


@pytest.mark.parametrize("n,p,seed", [(10, 0.3, 1), (10, 0.3, 2), (64, 0.05, 11), (254, 0.3, 5),
                                      (300, 0.01, 8), (3, 0.0, 1), (50, 1.0, 2)])
def test_exact_topology_matches_oracle(gossip, oracle, n, p, seed):
    t = gossip.Topology.gnp(n, p, seed, gossip.TOPO_EXACT)
    a, b = t.links()
    r = oracle.run_reference(num_nodes=n, connection_prob=p, sim_time_s=5.2, topo_seed=seed)
    assert np.array_equal(a, r.links[0]) and np.array_equal(b, r.links[1])
    peers, sockets = t.degrees()
    # Peer count / socket connections exactly as PrintStatistics reports them.
    assert np.array_equal(peers, r.peers)
    assert np.array_equal(sockets, r.sockets)


def test_fixup_is_no_forward_link_not_isolated(gossip):
    # p = 0: no sampled link; row 0 -> (0,1), row i -> (i,i-1).  The keys (0,1) and (1,0)
    # are parallel links, so nodes 0 and 1 see each other twice (multiplicity 2).
    t = gossip.Topology.gnp(5, 0.0, 1, gossip.TOPO_EXACT)
    a, b = t.links()
    assert list(zip(a.tolist(), b.tolist())) == [(0, 1), (1, 0), (2, 1), (3, 2), (4, 3)]
    peers, sockets = t.degrees()
    assert peers.tolist() == [2, 3, 2, 2, 1]
    assert sockets.tolist() == [1, 2, 2, 2, 1]
    rp, col, mult = t.csr()
    assert rp.tolist() == [0, 1, 3, 5, 7, 8]
    assert col.tolist() == [1, 0, 2, 1, 3, 2, 4, 3]
    assert mult.tolist() == [2, 2, 1, 1, 1, 1, 1, 1]


def test_last_node_always_gets_fixup(gossip):
    # Row n-1 has no j > i, so the key (n-1, n-2) always exists: with (n-2, n-1) sampled the
    # pair is a parallel link.
    for seed in range(1, 20):
        t = gossip.Topology.gnp(12, 0.9, seed, gossip.TOPO_EXACT)
        a, b = t.links()
        keys = set(zip(a.tolist(), b.tolist()))
        assert (11, 10) in keys
        peers, sockets = t.degrees()
        if (10, 11) in keys:
            rp, col, mult = t.csr()
            row = slice(rp[11], rp[12])
            assert mult[row][col[row] == 10].tolist() == [2]


def test_n_below_two_is_rejected(gossip):
    # p2pnetwork.cc:82 calls nodes.Get(1) for row 0 when n == 1: the reference aborts.
    with pytest.raises(gossip.GossipError):
        gossip.Topology.gnp(1, 0.3, 1)
    with pytest.raises(gossip.GossipError):
        gossip.P2PGossipNetworkSimulation(1)


def test_two_nodes_always_parallel(gossip):
    for seed in range(1, 6):
        t = gossip.Topology.gnp(2, 0.5, seed)
        peers, sockets = t.degrees()
        assert peers.tolist() == [2, 2] and sockets.tolist() == [1, 1]


def test_python_restatement_agrees(gossip):
    t = gossip.Topology.gnp(30, 0.2, 77)
    a, b = t.links()
    assert list(zip(a.tolist(), b.tolist())) == refrng.topology_links(30, 0.2, 77)


def test_skip_topology_law_and_fixup(gossip):
    n, p = 20000, 16.0 / 19999
    t = gossip.Topology.gnp(n, p, 3, gossip.TOPO_SKIP, threads=4)
    a, b = t.links()
    fwd = a < b
    # E[forward links] = p * n(n-1)/2; 5-sigma band.
    mean = p * n * (n - 1) / 2
    assert abs(int(fwd.sum()) - mean) < 5 * np.sqrt(mean)
    # Fix-up rule: every row has >= 1 key with that row as first element.
    assert np.array_equal(np.unique(a), np.arange(n))
    rows_with_forward = set(np.unique(a[fwd]).tolist())
    # Forward keys (a < b) other than the row-0 fix-up (0, 1) are sampled links; the fix-up
    # keys are (i, i-1), or (0, 1) for row 0, exactly for rows without a sampled j > i.
    fix = ~fwd
    fa, fb = a[fix], b[fix]
    assert np.all(fb == fa - 1)
    fix_rows = set(fa.tolist())
    if 0 not in rows_with_forward:
        # row 0's fix-up (0,1) looks like a forward key; it must be its only key
        assert a.tolist().count(0) == 1 and b[a == 0].tolist() == [1]
        rows_with_forward.discard(0)
        fix_rows.add(0)
    assert fix_rows == set(range(n)) - rows_with_forward
    assert n - 1 in fix_rows


def test_skip_topology_thread_invariant(gossip):
    t1 = gossip.Topology.gnp(5000, 0.003, 9, gossip.TOPO_SKIP, threads=1)
    t8 = gossip.Topology.gnp(5000, 0.003, 9, gossip.TOPO_SKIP, threads=8)
    for x, y in zip(t1.links(), t8.links()):
        assert np.array_equal(x, y)


def test_from_links_map_semantics(gossip):
    # Duplicate keys collapse (std::map), (a,b) and (b,a) are distinct keys.
    t = gossip.Topology.from_links(4, [2, 0, 0, 1, 3], [1, 1, 1, 0, 2])
    a, b = t.links()
    assert list(zip(a.tolist(), b.tolist())) == [(0, 1), (1, 0), (2, 1), (3, 2)]
    peers, sockets = t.degrees()
    assert peers.tolist() == [2, 3, 2, 1]
