"""Parity of the HIP engine (libgossip.so on an MI355X) with ORACLE A.

Bit-exact per-node counters (integer work); first-contact tick and hop count per
(node, shareId) against the oracle's event times (tick = floor(t / Latency)).
"""
import numpy as np
import pytest

import golden_util as G
from cases import CASES, L, T0

pytestmark = pytest.mark.gpu

STATS = ("gen", "recv", "fwd", "sent", "processed", "peers", "sockets")


def _engine_for(gossip, topo, events, latency_ns, t_cut, snapshots=(), flags=0, options=(), **kw):
    eng = gossip.Engine(topo.num_nodes, latency_ns, T0, t_cut, flags=flags, **kw)
    for k, v in options:
        eng.set_option(k, v)
    eng.set_topology(topo)
    for s in snapshots:
        eng.add_snapshot(s)
    eng.set_schedule(events)
    eng.run()
    eng.sync()
    return eng


@pytest.mark.parametrize("c", CASES, ids=[c["name"] for c in CASES])
def test_hand_cases(gossip, c):
    a = [x for x, _ in c["links"]]
    b = [y for _, y in c["links"]]
    topo = gossip.Topology.from_links(c["n"], a, b)
    ev = np.array(c["events"], dtype=np.int64)
    events = gossip.events_from_arrays(ev[:, 0], ev[:, 1], ev[:, 2])
    eng = _engine_for(gossip, topo, events, L, c["t_cut"])
    st = eng.stats()
    for k, want in c["expect"].items():
        assert getattr(st, k).tolist() == want, (k, getattr(st, k))
    assert np.array_equal(st.fwd, st.recv)


@pytest.mark.parametrize("name", G.names())
def test_golden_parity(gossip, name):
    g = G.load(name)
    p = g["params"]
    n = p["num_nodes"]
    sim = gossip.P2PGossipNetworkSimulation(n, topo_seed=p["topo_seed"], node_seed=p["node_seed"],
                                            topology_kind=gossip.TOPO_EXACT)
    if p.get("id_mask"):
        # the id_mask test knob lives in the schedule builder: drive the engine directly
        topo = gossip.Topology.gnp(n, p["connection_prob"], p["topo_seed"], gossip.TOPO_EXACT)
        lat = gossip.milliseconds_to_ns(p["latency_ms"])
        t_cut = gossip.seconds_to_ns(p["sim_time_s"] - 0.1)
        ev = gossip.make_schedule(n, p["node_seed"], T0, t_cut, id_mask=p["id_mask"])
        st = _engine_for(gossip, topo, ev, lat, t_cut).stats()
    else:
        sim.CreateRandomTopology(p["connection_prob"], p["latency_ms"])
        st = sim.Start(p["sim_time_s"])
        per = [(gossip.seconds_to_ns(t), gg, pp, s) for t, gg, pp, s in sim.periodic]
        assert np.array_equal(np.array(per, np.int64).reshape(-1, 4), g["periodic"])
    for k in STATS:
        assert np.array_equal(getattr(st, k), g[k]), k
    assert int(st.sent.sum()) == int(g["edge_events"])


def test_report_text_matches_oracle(gossip, oracle):
    sim = gossip.P2PGossipNetworkSimulation(10, topo_seed=11, node_seed=42)
    sim.CreateRandomTopology(0.3, 5.0)
    sim.Start(60.0)
    r = oracle.run_reference(num_nodes=10, connection_prob=0.3, sim_time_s=60.0, topo_seed=11,
                             node_seed=42)
    ost = gossip.Stats(r.gen, r.recv, r.fwd, r.sent, r.processed, r.peers, r.sockets)
    assert sim.PrintStatistics() == gossip.format_statistics(ost)
    want = "".join(gossip.format_periodic(t / 1e9, 10, g, p, s) for t, g, p, s in r.periodic)
    assert sim.PrintPeriodicStats() == want


# Pull variants: the defaults (k_pull over tile lists with saturation bits, dense-row tiles by the
# layer model), passes over consecutive words (no tile lists: no saturation bits, no dense rows),
# and dense rows forced on every listed tile.
KERNELS = {"auto": (), "no_tile_lists": (("pull_tiles", 0),), "dense_rows": (("dense_rows", 1),)}


def _trace_parity(gossip, oracle, n, p, seed, sim_time, lat_ms, kind=None, id_mask=0, kflags=0, options=()):
    kind = gossip.TOPO_EXACT if kind is None else kind
    topo = gossip.Topology.gnp(n, p, seed, kind)
    lat = gossip.milliseconds_to_ns(lat_ms)
    t_cut = gossip.seconds_to_ns(sim_time - 0.1)
    ev = gossip.make_schedule(n, seed + 1, T0, t_cut, id_mask=id_mask)
    eng = _engine_for(gossip, topo, ev, lat, t_cut, flags=gossip.F_TRACE | kflags, options=options)
    st = eng.stats()
    a, b = topo.links()
    r = oracle.run_replay(n, lat, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"], trace=True)
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(r, k)), k
    node, sid, tick, hop, via = eng.trace()
    tn, ti, tt, th, tv = r.trace
    ek = np.lexsort((sid, node))
    ok = np.lexsort((ti, tn))
    assert np.array_equal(node[ek], tn[ok]) and np.array_equal(sid[ek], ti[ok])
    assert np.array_equal(tick[ek], tt[ok] // lat)   # first-contact tick
    assert np.array_equal(hop[ek], th[ok])           # first-arrival hop count
    assert np.array_equal(via[ek], tv[ok])


@pytest.mark.parametrize("kern", list(KERNELS))
def test_trace_parity_sparse_4096(gossip, oracle, kern):
    _trace_parity(gossip, oracle, 4096, 16.0 / 4095, 21, 6.0, 5.0, options=KERNELS[kern])


@pytest.mark.parametrize("kern", list(KERNELS))
def test_trace_parity_dense_512(gossip, oracle, kern):
    _trace_parity(gossip, oracle, 512, 0.3, 22, 8.0, 5.0, options=KERNELS[kern])


@pytest.mark.parametrize("kern", list(KERNELS))
def test_trace_parity_collisions(gossip, oracle, kern):
    # 0x3FF id mask: dozens of generations per id, id groups of up to ~6 sources
    _trace_parity(gossip, oracle, 400, 0.01, 23, 15.0, 5.0, id_mask=0x3FF, options=KERNELS[kern])


@pytest.mark.parametrize("kern", list(KERNELS))
def test_trace_parity_odd_latency(gossip, oracle, kern):
    _trace_parity(gossip, oracle, 300, 0.02, 24, 10.37, 2.3, options=KERNELS[kern])


# Saturation bits and dense-row tiles (pull_kernel.h) against the oracle's counters and traces:
# forced dense rows on every listed tile (every k_pull row written, read without occupancy words),
# saturation bits off / on, where id groups (collisions: births landing in old tiles, whose sat
# bits must not be trusted), odd latencies (the in-tick cut: keep masks) and tile reuse happen.
SAT_DR = {"dr_forced": (("dense_rows", 1),), "dr_forced_nosat": (("dense_rows", 1), ("pull_sat", 0)),
          "sat_only": (("dense_rows", 0),), "both_off": (("dense_rows", 0), ("pull_sat", 0))}


@pytest.mark.parametrize("opts", list(SAT_DR))
def test_sat_dense_rows_collisions(gossip, oracle, opts):
    _trace_parity(gossip, oracle, 400, 0.01, 23, 15.0, 5.0, id_mask=0x3FF, options=SAT_DR[opts])


@pytest.mark.parametrize("opts", list(SAT_DR))
def test_sat_dense_rows_odd_latency_wide(gossip, oracle, opts):
    _trace_parity(gossip, oracle, 3000, 8.0 / 2999, 27, 6.37, 2.3, kind=gossip.TOPO_SKIP,
                  kflags=gossip.F_TILE_PER_TICK, options=SAT_DR[opts])


@pytest.mark.parametrize("opts", list(SAT_DR))
def test_sat_dense_rows_sparse_4096(gossip, oracle, opts):
    _trace_parity(gossip, oracle, 4096, 16.0 / 4095, 21, 6.0, 5.0, options=SAT_DR[opts])


@pytest.mark.parametrize("n,p,id_mask,sim", [(512, 0.3, 0, 8.0), (300, 0.05, 0xFFF, 30.0),
                                             (1000, 0.02, 0, 12.0)])
def test_dense_mfma_mode_matches_oracle(gossip, oracle, n, p, id_mask, sim):
    # GOSSIP_MODE_DENSE: the same tick engine with the int8-MFMA contraction as the pull.
    topo = gossip.Topology.gnp(n, p, 51, gossip.TOPO_EXACT)
    t_cut = gossip.seconds_to_ns(sim - 0.1)
    ev = gossip.make_schedule(n, 52, T0, t_cut, id_mask=id_mask)
    eng = _engine_for(gossip, topo, ev, L, t_cut, mode=gossip.MODE_DENSE, flags=gossip.F_TRACE)
    st = eng.stats()
    a, b = topo.links()
    r = oracle.run_replay(n, L, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"], trace=True)
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(r, k)), k
    node, sid, tick, hop, via = eng.trace()
    tn, ti, tt, th, tv = r.trace
    ek, ok = np.lexsort((sid, node)), np.lexsort((ti, tn))
    assert np.array_equal(tick[ek], tt[ok] // L) and np.array_equal(hop[ek], th[ok])
    assert eng.counters().dense_ops > 0


@pytest.mark.parametrize("kern", list(KERNELS))
def test_work_skipping_changes_nothing(gossip, kern):
    # Dead-word / saturated-node / empty-row skipping only removes reads that cannot add a
    # bit: the dense pull (F_NOSKIP) must give identical counters, with collisions in play.
    n = 6000
    topo = gossip.Topology.gnp(n, 10.0 / (n - 1), 41, gossip.TOPO_SKIP)
    t_cut = gossip.seconds_to_ns(8.0)
    ev = gossip.make_schedule(n, 5, T0, t_cut, id_mask=0x3FFF)
    a = _engine_for(gossip, topo, ev, L, t_cut, options=KERNELS[kern]).stats()
    b = _engine_for(gossip, topo, ev, L, t_cut, flags=gossip.F_NOSKIP, options=KERNELS[kern]).stats()
    for k in STATS:
        assert np.array_equal(getattr(a, k), getattr(b, k)), k


def test_wide_window_kernels_agree(gossip, oracle):
    # A window far wider than 64 words (a fresh tile every tick): every pull kernel, and the
    # production instantiation k_pull<32, 1, true> (non-temporal rows) with and without young-tile
    # slots, must match the oracle bit for bit.
    n = 3000
    topo = gossip.Topology.gnp(n, 6.0 / (n - 1), 43, gossip.TOPO_SKIP)
    t_cut = gossip.seconds_to_ns(5.7)
    ev = gossip.make_schedule(n, 7, T0, t_cut)
    a, b = topo.links()
    r = oracle.run_replay(n, L, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"])
    runs = [dict(o) for o in KERNELS.values()]
    runs += [{"pull_nt": 1}, {"pull_nt": 1, "young": 1, "young_nt": 1, "pull_grid": 16384},
             {"pull_nt": 1, "dense_rows": 1}, {"pull_nt": 1, "pull_sat": 0, "dense_rows": 0}]
    for opts in runs:
        eng = gossip.Engine(n, L, T0, t_cut, flags=gossip.F_TILE_PER_TICK)
        for k, v in opts.items():
            eng.set_option(k, v)
        eng.set_topology(topo)
        eng.set_schedule(ev)
        eng.run()
        eng.sync()
        st, c = eng.stats(), eng.counters()
        eng.close()
        assert c.words_hw > 64
        if opts.get("pull_nt"):
            assert c.pull_nt == 1 and c.pull_lpw == 32, opts  # k_pull<32, 1, true>
        for k in STATS:
            assert np.array_equal(getattr(st, k), getattr(r, k)), (opts, k)


def test_tile_list_options_agree(gossip, oracle):
    # k_pull's pass -> tile lists (pull_tiles) and their age order (pull_tile_order) only change
    # which lanes serve which tiles: a wide window of tiles of every age (a fresh tile per tick),
    # id collisions in play, must give the oracle's counters and trace under every setting.
    n = 3000
    topo = gossip.Topology.gnp(n, 8.0 / (n - 1), 45, gossip.TOPO_SKIP)
    t_cut = gossip.seconds_to_ns(6.3)
    ev = gossip.make_schedule(n, 9, T0, t_cut, id_mask=0xFFF)
    a, b = topo.links()
    r = oracle.run_replay(n, L, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"], trace=True)
    tn, ti, tt, th, tv = r.trace
    ok = np.lexsort((ti, tn))
    prod = {"pull_nt": 1, "pull_grid": 16384, "pull_tile_order": 1}  # the C4 bench's k_pull<32,1,true>
    for opts in ({}, {"pull_tile_order": 0}, {"pull_tiles": 0}, prod,
                 dict(prod, young=1, young_nt=1), dict(prod, young=1, young_nt=1, dense_rows=1),
                 dict(prod, dense_rows=1), dict(prod, dense_rows=1, pull_sat=0), {"pull_sat": 0, "dense_rows": 0}):
        eng = gossip.Engine(n, L, T0, t_cut, flags=gossip.F_TILE_PER_TICK | gossip.F_TRACE)
        for k, v in opts.items():
            eng.set_option(k, v)
        eng.set_topology(topo)
        eng.set_schedule(ev)
        eng.run()
        eng.sync()
        st, c = eng.stats(), eng.counters()
        assert c.words_hw > 64 and (c.pull_tiles == 0 or opts.get("pull_tiles") != 0), opts
        if opts.get("pull_nt"):
            assert c.pull_nt == 1 and c.pull_lpw == 32 and c.pull_grid == 12, opts  # (3,000 nodes: 12 blocks)
        if opts.get("young"):
            assert c.young_launches > 0, opts
        for k in STATS:
            assert np.array_equal(getattr(st, k), getattr(r, k)), (opts, k)
        node, sid, tick, hop, via = eng.trace()
        ek = np.lexsort((sid, node))
        assert np.array_equal(node[ek], tn[ok]) and np.array_equal(sid[ek], ti[ok]), opts
        assert np.array_equal(tick[ek], tt[ok] // L) and np.array_equal(via[ek], tv[ok]), opts
        eng.close()


def test_window_growth_is_transparent(gossip, oracle):
    # Start with a one-tile window: the engine must widen its rows mid-run and stay exact.
    n = 3000
    topo = gossip.Topology.gnp(n, 8.0 / (n - 1), 42, gossip.TOPO_SKIP)
    t_cut = gossip.seconds_to_ns(7.0)
    ev = gossip.make_schedule(n, 6, T0, t_cut)
    eng = _engine_for(gossip, topo, ev, L, t_cut, max_words=16)
    st = eng.stats()
    assert eng.counters().words_cap > 16
    a, b = topo.links()
    r = oracle.run_replay(n, L, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"])
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(r, k)), k


def test_early_retire_near_capacity(gossip, oracle):
    # A window sized to the run's own peak: near its capacity the allocator first retires tiles from
    # the last tick's liveness (one tick earlier than the regular two-tick lag) instead of widening
    # the window -- results unchanged, no growth
    n = 3000
    topo = gossip.Topology.gnp(n, 8.0 / (n - 1), 42, gossip.TOPO_SKIP)
    t_cut = gossip.seconds_to_ns(7.0)
    ev = gossip.make_schedule(n, 6, T0, t_cut)
    free = _engine_for(gossip, topo, ev, L, t_cut, flags=gossip.F_TILE_PER_TICK)
    peak = free.counters().words_hw
    free.close()
    eng = _engine_for(gossip, topo, ev, L, t_cut, flags=gossip.F_TILE_PER_TICK, max_words=peak)
    st, c = eng.stats(), eng.counters()
    eng.close()
    assert c.window_early_retires > 0 and c.words_cap == peak and c.words_hw <= peak
    a, b = topo.links()
    r = oracle.run_replay(n, L, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"])
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(r, k)), k


@pytest.mark.parametrize("rule", ["hash", "birth_tick", "birth_tick_fresh_tiles"])
def test_sharded_engines_sum_to_whole(gossip, rule):
    n = 5000
    topo = gossip.Topology.gnp(n, 12.0 / (n - 1), 31, gossip.TOPO_SKIP)
    t_cut = gossip.seconds_to_ns(9.9)
    ev = gossip.make_schedule(n, 77, T0, t_cut, id_mask=0xFFFF)
    whole = _engine_for(gossip, topo, ev, L, t_cut).stats()
    # (bench.shard_flags: the birth-tick rule runs with a fresh tile per birth tick)
    fl = {"hash": 0, "birth_tick": gossip.F_SHARD_BY_TICK,
          "birth_tick_fresh_tiles": gossip.F_SHARD_BY_TICK | gossip.F_TILE_PER_TICK}[rule]
    parts = [_engine_for(gossip, topo, ev, L, t_cut, flags=fl, shard_rank=r, shard_count=3).stats()
             for r in range(3)]
    for k in ("gen", "recv", "fwd", "sent", "processed"):
        tot = sum(getattr(s, k).astype(np.uint64) for s in parts)
        assert np.array_equal(tot, getattr(whole, k).astype(np.uint64)), k
    owner = gossip.shard_events(topo, ev, 3, by_tick_latency_ns=L if fl & gossip.F_SHARD_BY_TICK else 0)
    for r in range(3):
        assert np.array_equal(np.bincount(ev["node"][owner == r], minlength=n), parts[r].gen)


def test_large_sparse_invariants(gossip):
    # 1M nodes, average degree 16 (C3's graph), the first 40 ticks after t = 5 s.
    n = 1_000_000
    topo = gossip.Topology.gnp(n, 16.0 / (n - 1), 3, gossip.TOPO_SKIP, threads=16)
    t_cut = gossip.seconds_to_ns(59.9)
    ev = gossip.make_schedule(n, 1000, T0, t_cut, t_gen_end_ns=T0 + 40 * L, threads=16)
    eng = gossip.Engine(n, L, T0, t_cut)
    eng.set_topology(topo)
    eng.set_schedule(ev)
    eng.run(eng.first_tick + 40)
    st = eng.stats()
    c = eng.counters()
    assert np.array_equal(st.fwd, st.recv)
    assert np.array_equal(st.sent, st.peers.astype(np.uint64) * (st.gen + st.recv))
    if len(np.unique(ev["share_id"])) == len(ev):
        assert np.array_equal(st.processed, st.gen + st.recv)
    else:
        assert np.all(st.processed <= st.gen + st.recv)
    assert c.edge_events == int(st.sent.sum())
    assert int(st.gen.sum()) == len(ev)
    # a share born in the first ticks has flooded its component by tick 40
    assert int(st.recv.max()) > 0


def test_parity_65536_sparse(gossip, oracle):
    # SURVEY §7 minimum slice: a 65,536-node seeded case bit-exact, floods run to completion
    # (the generations of the first tick after t_start; every id unique at this size).
    n = 65536
    topo = gossip.Topology.gnp(n, 16.0 / (n - 1), 61, gossip.TOPO_SKIP)
    t_cut = gossip.seconds_to_ns(5.5)
    ev = gossip.make_schedule(n, 62, T0, t_cut, t_gen_end_ns=T0 + L)
    assert len(ev) > 10
    eng = _engine_for(gossip, topo, ev, L, t_cut, flags=gossip.F_TRACE)
    st = eng.stats()
    a, b = topo.links()
    r = oracle.run_replay(n, L, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"], trace=True)
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(r, k)), k
    node, sid, tick, hop, via = eng.trace()
    tn, ti, tt, th, tv = r.trace
    ek, ok = np.lexsort((sid, node)), np.lexsort((ti, tn))
    assert np.array_equal(node[ek], tn[ok]) and np.array_equal(sid[ek], ti[ok])
    assert np.array_equal(tick[ek], tt[ok] // L) and np.array_equal(hop[ek], th[ok])
    assert int(st.recv.sum()) > n  # the floods covered the graph


# Push marks (round 6, option pull_push, pull_kernel.h): rows of push-write tiles mark their
# writers' peers, and the next tick's k_pull skips push tiles at unmarked nodes.  Forced on every
# listed tile that is not dense-row (1) -- so tiles at every hop, with births landing in old tiles
# (collisions: packed tiles), keep masks (the in-tick cut of an odd latency) and young tiles beside
# -- the counters and traces must equal the oracle's; auto (-1) picks the tiles by the layer model.
PUSH = {"forced": {"pull_push": 1}, "forced_young": {"pull_push": 1, "young": 1},
        "forced_dense_rows": {"pull_push": 1, "dense_rows": 1}, "forced_nt": {"pull_push": 1, "pull_nt": 1},
        "auto": {"pull_push": -1}, "off": {"pull_push": 0}}


@pytest.mark.parametrize("case,opts", [(c, o) for c in ("wide_collisions", "odd_latency_cut", "packed_tiles")
                                        for o in ("forced", "forced_young", "auto")] +
                         [("packed_tiles", "forced_dense_rows"), ("wide_collisions", "forced_nt"),
                          ("packed_tiles", "off")])
def test_push_marks(gossip, oracle, case, opts):
    n, deg, seed, sim, lat_ms, id_mask, fl = {
        "wide_collisions": (3000, 8.0, 45, 6.3, 5.0, 0xFFF, gossip.F_TILE_PER_TICK),
        "odd_latency_cut": (3000, 8.0, 27, 6.37, 2.3, 0, gossip.F_TILE_PER_TICK),
        "packed_tiles": (4096, 16.0, 21, 6.0, 5.0, 0x3FFF, 0)}[case]
    topo = gossip.Topology.gnp(n, deg / (n - 1), seed, gossip.TOPO_SKIP)
    lat = gossip.milliseconds_to_ns(lat_ms)
    t_cut = gossip.seconds_to_ns(sim - 0.1)
    ev = gossip.make_schedule(n, seed + 1, T0, t_cut, id_mask=id_mask)
    eng = _engine_for(gossip, topo, ev, lat, t_cut, flags=gossip.F_TRACE | fl, options=tuple(PUSH[opts].items()))
    st, c = eng.stats(), eng.counters()
    a, b = topo.links()
    r = oracle.run_replay(n, lat, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"], trace=True)
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(r, k)), k
    node, sid, tick, hop, via = eng.trace()
    tn, ti, tt, th, tv = r.trace
    ek, ok = np.lexsort((sid, node)), np.lexsort((ti, tn))
    assert np.array_equal(node[ek], tn[ok]) and np.array_equal(sid[ek], ti[ok])
    assert np.array_equal(tick[ek], tt[ok] // lat) and np.array_equal(hop[ek], th[ok])
    assert np.array_equal(via[ek], tv[ok])
    if opts == "off":
        assert c.pull_push_tiles == 0 and c.pull_marks == 0
    elif opts in ("forced", "forced_young", "forced_nt") and c.pull_lpw == 32:
        # (push marks run in k_pull<32, 1, .., SP>; with dense rows forced every tile but the
        # freshest is dense-row, and a fresh tile got births the tick before: never a push tile)
        assert c.pull_pushw_tiles > 0 and c.pull_push_tiles > 0 and c.pull_marks > 0, c.pull_lpw
    eng.close()
