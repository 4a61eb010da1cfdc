"""Pin ORACLE A (and the product host code) to the published algorithms it restates.

The reference ships no tests or golden vectors, so the oracle is pinned
by known-answer tests of the primitives it shares with the reference and by an independent
pure-Python restatement (tests/refrng.py) of the reference's topology and schedule rules.
"""
import random

import numpy as np
import pytest

import refrng


def test_mt19937_kat():
    # C++11 [rand.predef]: the 10000th consecutive invocation of a default-constructed
    # std::mt19937 produces 4123659995.
    g = refrng.MT19937()
    x = None
    for _ in range(10000):
        x = g()
    assert x == 4123659995


def test_time_conversion_known_values(oracle, gossip):
    # 2**-10 s = 976562.5 ns exactly: ns-3's int64x64 Round() is half-up (not half-even).
    cases = {59.9: 59_900_000_000, 5.0: 5_000_000_000, 0.1: 100_000_000, 60.0 - 0.1: 59_900_000_000,
             1e-9: 1, 2.0 ** -10: 976_563, 3 * 2.0 ** -10: 2_929_688}
    for x, ns in cases.items():
        assert refrng.seconds_to_ns(x) == ns, x
        assert oracle.seconds_to_ns(x) == ns, x
        assert gossip.seconds_to_ns(x) == ns, x
    assert oracle.milliseconds_to_ns(5.0) == 5_000_000
    assert gossip.milliseconds_to_ns(3.7) == 3_700_000


def test_time_conversion_random_exact(oracle, gossip):
    rng = random.Random(7)
    for _ in range(3000):
        x = rng.uniform(2.0, 5.0)
        want = refrng.seconds_to_ns(x)
        assert oracle.seconds_to_ns(x) == want
        assert gossip.seconds_to_ns(x) == want


@pytest.mark.parametrize("n,p,seed", [(10, 0.3, 1), (17, 0.1, 99), (40, 0.05, 3), (2, 0.5, 4)])
def test_oracle_topology_matches_python_restatement(oracle, n, p, seed):
    r = oracle.run_reference(num_nodes=n, connection_prob=p, sim_time_s=5.5, topo_seed=seed)
    got = list(zip(r.links[0].tolist(), r.links[1].tolist()))
    assert got == refrng.topology_links(n, p, seed)


@pytest.mark.parametrize("node_seed", [1000, 4294967290])
def test_oracle_schedule_matches_python_restatement(oracle, node_seed):
    n = 6
    r = oracle.run_reference(num_nodes=n, sim_time_s=30.0, node_seed=node_seed)
    ns, node, ids = r.gen_events
    t_cut = refrng.seconds_to_ns(30.0 - 0.1)
    for v in range(n):
        want = refrng.node_schedule(v, node_seed, 5_000_000_000, t_cut)
        sel = node == v
        got = list(zip(ns[sel].tolist(), ids[sel].tolist()))
        assert got == want


def test_share_id_formula_and_hash_identity(oracle):
    # GenerateUniqueShareId (p2pnode.cc:203-208): (uint32)(id*1e6 + g*1e3 + ns%1000) with
    # std::hash<uint64_t> the identity (libstdc++ functional_hash.h:169).
    r = oracle.run_reference(num_nodes=5, sim_time_s=40.0)
    ns, node, ids = r.gen_events
    for v in range(5):
        sel = np.flatnonzero(node == v)
        for g, k in enumerate(sel):
            assert ids[k] == (v * 1_000_000 + g * 1000 + int(ns[k]) % 1000) & 0xFFFFFFFF
