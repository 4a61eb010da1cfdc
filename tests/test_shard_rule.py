"""Share-shard rules (gossip_shard_events, gossip_shard_events_by_tick; CPU only).

Shares are independent floods except inside an id instance -- the generations that share one id
within one connected component share one seen-set entry (p2pnode.cc:189) -- so a rule may split
the instances over shards any way it likes as long as every instance stays whole.  The birth-tick
rule (GOSSIP_F_SHARD_BY_TICK) gives an instance to shard (tick of its first generation) mod S."""
import os

import numpy as np
from scipy.sparse import csr_matrix
from scipy.sparse.csgraph import connected_components

L = 5_000_000
T0 = 5_000_000_000


def _workload(gossip):
    n = 3000
    topo = gossip.Topology.gnp(n, 1.2 / (n - 1), 17, gossip.TOPO_SKIP)
    ev = gossip.make_schedule(n, 18, T0, gossip.seconds_to_ns(40.0), id_mask=0x7FF)
    rp, col, _ = topo.csr()
    m = csr_matrix((np.ones(len(col)), col, rp), shape=(n, n))
    ncomp, comp = connected_components(m, directed=False)
    return topo, ev, comp, ncomp


def test_birth_tick_rule_keeps_instances_whole(gossip):
    topo, ev, comp, ncomp = _workload(gossip)  # (the fix-up links usually leave one component)
    ids, counts = np.unique(ev["share_id"], return_counts=True)
    assert (counts > 1).sum() > 100  # plenty of colliding ids
    for S in (2, 3, 8):
        owner = gossip.shard_events(topo, ev, S, by_tick_latency_ns=L)
        key = ev["share_id"].astype(np.uint64) << np.uint64(32) | comp[ev["node"]].astype(np.uint64)
        lone = np.isin(ev["share_id"], ids[counts == 1])
        # every instance whole, on the shard of its first generation's tick
        order = np.lexsort((ev["ns"], key))
        k, o, ns = key[order], owner[order], ev["ns"][order]
        start = np.r_[True, k[1:] != k[:-1]]
        first_ns = np.maximum.accumulate(np.where(start, np.arange(len(k)), 0))
        assert np.array_equal(o, o[first_ns]), S
        assert np.array_equal(o, (ns[first_ns] // L % S).astype(o.dtype)), S
        # a lone id: the tick of its one generation
        assert np.array_equal(owner[lone], (ev["ns"][lone] // L % S).astype(owner.dtype))
        # the hash rule keeps instances whole too, and differs
        h = gossip.shard_events(topo, ev, S)
        assert np.array_equal(h[order], h[order][first_ns])
        assert not np.array_equal(h, owner)


def test_birth_tick_rule_fills_a_shard_per_tick(gossip):
    # distinct ids: each tick's generations all go to one shard, the shards take turns
    n = 5000
    topo = gossip.Topology.gnp(n, 8.0 / (n - 1), 19, gossip.TOPO_SKIP)
    ev = gossip.make_schedule(n, 20, T0, gossip.seconds_to_ns(8.0))
    assert len(np.unique(ev["share_id"])) == len(ev)
    owner = gossip.shard_events(topo, ev, 4, by_tick_latency_ns=L)
    tick = ev["ns"] // L
    for t in np.unique(tick):
        assert len(np.unique(owner[tick == t])) == 1
    assert np.array_equal(np.bincount(owner, minlength=4) > 0, [True] * 4)


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_auto_rule_takes_birth_ticks_from_8_shards():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert [bench.resolve_shard_rule("auto", s) for s in (1, 2, 4, 8, 16)] == ["hash", "hash", "hash", "tick", "tick"]
    assert bench.resolve_shard_rule("hash", 8) == "hash" and bench.resolve_shard_rule("tick", 2) == "tick"
    # the birth-tick rule opens a fresh tile per birth tick; the hash rule packs tiles
    assert bench.shard_flags("tick") == bench.gossip.F_SHARD_BY_TICK | bench.gossip.F_TILE_PER_TICK
    assert bench.shard_flags("hash") == 0
    assert bench.shard_flags("hash", "on") == bench.gossip.F_TILE_PER_TICK
    assert bench.shard_flags("tick", "off") == bench.gossip.F_SHARD_BY_TICK
