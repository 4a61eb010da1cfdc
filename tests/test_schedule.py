"""Share-generation schedule (product host code) vs the oracle.

Reference: P2PNode seeding p2pnode.cc:33-43, ScheduleNextShare :97-104,
GenerateAndGossipShare :106-125 (peers.empty() branch before t=5 s), GenerateUniqueShareId
:201-209, run window p2pnetwork.cc:193-218.
"""
import numpy as np
import pytest

import refrng


@pytest.mark.parametrize("n,sim,seed", [(10, 60.0, 1000), (37, 20.0, 5), (5, 9.0, 4294967295)])
def test_schedule_matches_oracle(gossip, oracle, n, sim, seed):
    t_start = gossip.seconds_to_ns(5.0)
    t_cut = gossip.seconds_to_ns(sim - 0.1)
    ev = gossip.make_schedule(n, seed, t_start, t_cut)
    r = oracle.run_reference(num_nodes=n, sim_time_s=sim, node_seed=seed)
    ons, onode, oid = r.gen_events
    o = np.lexsort((onode, ons))
    assert np.array_equal(ev["ns"], ons[o])
    assert np.array_equal(ev["node"], onode[o])
    assert np.array_equal(ev["share_id"], oid[o])
    # PrintStatistics "Generated" column
    assert np.array_equal(np.bincount(ev["node"], minlength=n), r.gen)


def test_schedule_window_and_python_restatement(gossip):
    t_start = gossip.seconds_to_ns(5.0)
    t_cut = gossip.seconds_to_ns(30.0 - 0.1)
    ev = gossip.make_schedule(8, 123, t_start, t_cut)
    assert ev["ns"].min() >= t_start and ev["ns"].max() < t_cut
    assert np.all(np.diff(ev["ns"]) >= 0)
    for v in range(8):
        want = refrng.node_schedule(v, 123, t_start, t_cut)
        sel = ev["node"] == v
        assert list(zip(ev["ns"][sel].tolist(), ev["share_id"][sel].tolist())) == want


def test_schedule_thread_invariant_and_gen_end(gossip):
    t_start = gossip.seconds_to_ns(5.0)
    t_cut = gossip.seconds_to_ns(59.9)
    a = gossip.make_schedule(3000, 77, t_start, t_cut, threads=1)
    b = gossip.make_schedule(3000, 77, t_start, t_cut, threads=8)
    assert np.array_equal(a, b)
    end = gossip.seconds_to_ns(9.0)
    c = gossip.make_schedule(3000, 77, t_start, t_cut, t_gen_end_ns=end, threads=8)
    assert np.array_equal(c, a[a["ns"] < end])


def test_id_mask_forces_collisions(gossip):
    t_start = gossip.seconds_to_ns(5.0)
    t_cut = gossip.seconds_to_ns(59.9)
    full = gossip.make_schedule(50, 1, t_start, t_cut)
    masked = gossip.make_schedule(50, 1, t_start, t_cut, id_mask=0x3F)
    assert np.array_equal(masked["share_id"], full["share_id"] & 0x3F)
    assert len(np.unique(masked["share_id"])) < len(masked)


def test_no_collisions_below_threshold(gossip):
    # ids are collision-free for n <= 128,849 at simTime ~ 60 s.
    t_start = gossip.seconds_to_ns(5.0)
    t_cut = gossip.seconds_to_ns(59.9)
    ev = gossip.make_schedule(20000, 3, t_start, t_cut, threads=8)
    assert len(np.unique(ev["share_id"])) == len(ev)
