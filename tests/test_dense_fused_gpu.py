"""The fused DENSE pull (k_dense_fused, dense_kernel.h): one persistent kernel per tick does the
int8-MFMA contraction, the dedup against seen and writes the transposed frontier of the next tick
(with k_births), so no tick runs k_transpose / k_dense_bits / k_dense_dedup unless it must (id
groups, row partitions, the no-skip diagnostic).  Every test runs the fused path, the three-kernel
path (option dense_fused 0) and ORACLE A on the same inputs; counters and first-contact traces must
agree bit for bit (p2pnode.cc:127-199)."""
import numpy as np
import pytest

from cases import L, T0

pytestmark = pytest.mark.gpu

STATS = ("gen", "recv", "fwd", "sent", "processed", "peers", "sockets")


def _run(gossip, topo, ev, lat, t_cut, fused, flags=0, snapshots=(), **kw):
    eng = gossip.Engine(topo.num_nodes, lat, T0, t_cut, mode=gossip.MODE_DENSE, flags=flags, **kw)
    eng.set_option("dense_fused", 1 if fused else 0)
    eng.set_topology(topo)
    for s in snapshots:
        eng.add_snapshot(s)
    eng.set_schedule(ev)
    eng.run()
    eng.sync()
    out = (eng.stats(), eng.counters(), eng.trace() if flags & gossip.F_TRACE else None,
           [eng.snapshot(k) for k in range(len(snapshots))])
    eng.close()
    return out


def _check(gossip, oracle, n, p, seed, sim_time, lat_ms, id_mask=0, flags=0, snapshots=(), expect_all_fused=None, **kw):
    topo = gossip.Topology.gnp(n, p, seed, gossip.TOPO_EXACT)
    lat = gossip.milliseconds_to_ns(lat_ms)
    t_cut = gossip.seconds_to_ns(sim_time - 0.1)
    ev = gossip.make_schedule(n, seed + 1, T0, t_cut, id_mask=id_mask)
    flags |= gossip.F_TRACE
    fs, fc, ftr, fsn = _run(gossip, topo, ev, lat, t_cut, True, flags, snapshots, **kw)
    us, uc, utr, usn = _run(gossip, topo, ev, lat, t_cut, False, flags, snapshots, **kw)
    assert fc.dense_fused_launches > 0 and uc.dense_fused_launches == 0
    if expect_all_fused is True:
        assert fc.dense_fused_launches == fc.pull_launches, (fc.dense_fused_launches, fc.pull_launches)
    if expect_all_fused is False:  # id groups: some ticks take the three-kernel path
        assert 0 < fc.dense_fused_launches < fc.pull_launches
    for k in STATS:
        assert np.array_equal(getattr(fs, k), getattr(us, k)), ("fused vs three-kernel", k)
    assert fsn == usn
    assert fc.edge_events == uc.edge_events
    for a, b in zip(ftr, utr):
        assert np.array_equal(a, b)
    if flags & gossip.F_HOP_BATCH:
        return fs, fc
    a, b = topo.links()
    r = oracle.run_replay(n, lat, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"], trace=True)
    for k in STATS:
        assert np.array_equal(getattr(fs, k), getattr(r, k)), ("fused vs ORACLE A", k)
    node, sid, tick, hop, via = ftr
    tn, ti, tt, th, tv = r.trace
    ek, ok = np.lexsort((sid, node)), np.lexsort((ti, tn))
    assert np.array_equal(node[ek], tn[ok]) and np.array_equal(sid[ek], ti[ok])
    assert np.array_equal(tick[ek], tt[ok] // lat) and np.array_equal(hop[ek], th[ok])
    assert np.array_equal(via[ek], tv[ok])
    return fs, fc


def test_fused_one_stage(gossip, oracle):
    # n <= 1,024: one K stage, 4 row blocks of which the last is padding beyond n
    _check(gossip, oracle, 700, 0.3, 71, 7.0, 5.0, expect_all_fused=True)


def test_fused_many_stages_ragged_n(gossip, oracle):
    # n = 3,000: n_pad 3,072 (3 stages), the last row block ragged; p = 0.1 keeps floods ~3 hops
    _check(gossip, oracle, 3000, 0.1, 72, 5.4, 5.0, expect_all_fused=True)


def test_fused_odd_latency_cut_and_snapshots(gossip, oracle):
    # 2.3 ms ticks: the PrintStatistics cut falls inside a tick (keep masks) and the periodic
    # snapshots at non-tick-aligned times count through the snapshot masks
    snaps = [gossip.seconds_to_ns(t) for t in (5.6, 6.1)]
    _check(gossip, oracle, 1500, 0.2, 73, 6.37, 2.3, snapshots=snaps, expect_all_fused=True)


def test_fused_with_id_groups(gossip, oracle):
    # colliding ids: ticks whose window holds a group word run the three-kernel path, the others
    # fused -- the transposed frontier is rebuilt by k_transpose after every such tick
    _check(gossip, oracle, 600, 0.05, 74, 16.0, 5.0, id_mask=0xFFF, expect_all_fused=False)


def test_fused_window_growth(gossip, oracle):
    # a one-tile window and a fresh tile per tick: the rows widen mid-run (FT and stage masks
    # reallocated, the next tick's FT rebuilt by k_transpose)
    fs, fc = _check(gossip, oracle, 2000, 0.1, 75, 5.6, 5.0, flags=gossip.F_TILE_PER_TICK, max_words=16)
    assert fc.words_cap > 16


def test_fused_hop_batched_snapshots(gossip, oracle):
    # hop-batched (the C2 operating point: thousands of concurrent columns), periodic snapshots
    n = 2048
    snaps = [gossip.seconds_to_ns(t) for t in (10.0, 20.0)]
    fs, fc = _check(gossip, oracle, n, 0.3, 76, 25.0, 5.0, flags=gossip.F_HOP_BATCH, snapshots=snaps,
                    expect_all_fused=True)
    topo = gossip.Topology.gnp(n, 0.3, 76, gossip.TOPO_EXACT)
    t_cut = gossip.seconds_to_ns(24.9)
    ev = gossip.make_schedule(n, 77, T0, t_cut)
    a, b = topo.links()
    # (ORACLE B: 2,048 nodes x ~600 peers x ~8k shares is too many events for ORACLE A)
    r = oracle.run_oracle_b(n, L, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"], threads=16)
    for k in STATS:
        assert np.array_equal(getattr(fs, k), getattr(r, k)), k
    assert fc.words_hw >= 64  # > 16 column tiles in flight


@pytest.mark.parametrize("n,p,seed", [(1100, 0.1, 78), (2048, 0.3, 79)])
def test_fused_every_tile_split(gossip, oracle, monkeypatch, n, p, seed):
    # GOSSIP_DENSE_ROUNDS=0: no whole-tile rounds, every live tile goes through the load-balanced
    # tail, so most tiles are split between blocks and meet in the inc / ticket reduction
    # (dense_kernel.h split-tile path: each wave's atomics acknowledged before the ticket)
    monkeypatch.setenv("GOSSIP_DENSE_ROUNDS", "0")
    flags = gossip.F_HOP_BATCH if n == 2048 else 0
    _check(gossip, oracle, n, p, seed, 5.6 if not flags else 12.0, 5.0, flags=flags, expect_all_fused=True)
