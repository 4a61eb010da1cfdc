"""ORACLE A against hand-derived cases (tests/cases.py) and run-level invariants."""
import numpy as np
import pytest

from cases import CASES, L, T0


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_oracle_hand_cases(oracle, c):
    a = [x for x, _ in c["links"]]
    b = [y for _, y in c["links"]]
    ev = np.array(c["events"], dtype=np.int64)
    r = oracle.run_replay(c["n"], L, T0, c["t_cut"], a, b, ev[:, 0], ev[:, 1], ev[:, 2])
    for k, want in c["expect"].items():
        assert getattr(r, k).tolist() == want, (k, getattr(r, k))
    assert np.array_equal(r.fwd, r.recv)
    assert r.edge_events == int(r.sent.sum())


@pytest.mark.parametrize("n,p,seed", [(10, 0.3, 1), (60, 0.1, 2), (200, 0.02, 3)])
def test_oracle_invariants(oracle, n, p, seed):
    r = oracle.run_reference(num_nodes=n, connection_prob=p, sim_time_s=25.0, topo_seed=seed)
    assert np.array_equal(r.fwd, r.recv)
    # ideal model: every emission goes to all peers
    assert np.array_equal(r.sent, r.peers.astype(np.uint64) * (r.gen + r.recv))
    # no id collisions at these sizes: processed = gen + recv
    assert np.array_equal(r.processed, r.gen + r.recv)
    assert r.edge_events == int(r.sent.sum())
    # periodic totals are monotone and the last one is below the final totals
    gens = [g for _, g, _, _ in r.periodic]
    assert gens == sorted(gens) and gens[-1] <= int(r.gen.sum())


def test_register_delay_changes_only_early_sends(oracle):
    a = oracle.run_reference(num_nodes=20, connection_prob=0.2, sim_time_s=20.0)
    b = oracle.run_reference(num_nodes=20, connection_prob=0.2, sim_time_s=20.0,
                             register_delay_ns=15_000_000)
    assert np.array_equal(a.peers, b.peers) and np.array_equal(a.sockets, b.sockets)
    assert np.array_equal(a.gen, b.gen)
