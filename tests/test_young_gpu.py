"""Young-tile slots (k_pull_young, young_kernel.h) against ORACLE A.

Young tiles are switched on by default only for n >= 2^20 (C4; C3's 1,000,000 nodes are just
below); here they are forced on small
graphs, with a fresh tile every tick (so every tick has young, leaving and fresh tiles), tiny slot
capacities (so nodes overflow to dense rows, in the pull and in the births), every young age, and
forced id collisions (id-group births that must find or cancel arrivals inside slots).  Per-node
counters and the first-contact trace must equal the oracle's bit for bit.
"""
import numpy as np
import pytest

from cases import T0

pytestmark = pytest.mark.gpu

STATS = ("gen", "recv", "fwd", "sent", "processed", "peers", "sockets")


def _run(gossip, topo, ev, lat, t_cut, opts, flags=0, snapshots=()):
    eng = gossip.Engine(topo.num_nodes, lat, T0, t_cut, flags=flags)
    for k, v in opts.items():
        eng.set_option(k, v)
    eng.set_topology(topo)
    for s in snapshots:
        eng.add_snapshot(s)
    eng.set_schedule(ev)
    eng.run()
    eng.sync()
    return eng


def _parity(gossip, oracle, n, p, seed, sim_s, lat_ms, opts, id_mask=0, flags=0, trace=True):
    topo = gossip.Topology.gnp(n, p, seed, gossip.TOPO_SKIP if n > 5000 else gossip.TOPO_EXACT)
    lat = gossip.milliseconds_to_ns(lat_ms)
    t_cut = gossip.seconds_to_ns(sim_s - 0.1)
    ev = gossip.make_schedule(n, seed + 1, T0, t_cut, id_mask=id_mask)
    f = flags | (gossip.F_TRACE if trace else 0)
    eng = _run(gossip, topo, ev, lat, t_cut, dict(opts, young=1), flags=f)
    st = eng.stats()
    c = eng.counters()
    a, b = topo.links()
    r = oracle.run_replay(n, lat, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"], trace=trace)
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(r, k)), (opts, k)
    if trace:
        node, sid, tick, hop, via = eng.trace()
        tn, ti, tt, th, tv = r.trace
        ek, ok = np.lexsort((sid, node)), np.lexsort((ti, tn))
        assert np.array_equal(node[ek], tn[ok]) and np.array_equal(sid[ek], ti[ok])
        assert np.array_equal(tick[ek], tt[ok] // lat) and np.array_equal(hop[ek], th[ok])
        assert np.array_equal(via[ek], tv[ok])
    eng.close()
    return c


# (5 of the 9 cap x age pairs: overflow-heavy, mid and roomy slots at the short, mid and long
# ages -- keeps the -m gpu suite inside its time budget)
@pytest.mark.parametrize("cap,age", [(1, 3), (1, 6), (3, 3), (127, 1), (127, 6)])
def test_young_sparse_4096(gossip, oracle, cap, age):
    c = _parity(gossip, oracle, 4096, 16.0 / 4095, 71, 6.0, 5.0,
                dict(young_cap=cap, young_age=age), flags=gossip.F_TILE_PER_TICK)
    assert c.young_launches > 0 and c.young_slot_lines > 0
    if cap == 1 and age >= 3:
        assert c.young_fallback_rows > 0  # overflowed peers were read through dense rows


@pytest.mark.parametrize("cap,id_mask", [(3, 0), (127, 0), (127, 0x3FF)])
def test_young_seen_lists(gossip, oracle, cap, id_mask):
    # seen lists (young_kernel.h): a node's seen bits of its young tiles as list entries (read with
    # the peers' slots, applied as AND-NOT, whole groups), materialised into dense seen rows when a
    # tile leaves the young set -- no dense seen word is read while no list overflows
    c = _parity(gossip, oracle, 3000, 12.0 / 2999, 81, 6.0, 5.0,
                dict(young_cap=cap, young_age=4), id_mask=id_mask, flags=gossip.F_TILE_PER_TICK)
    assert c.young_list_lines > 0 and c.young_fresh_lines > 0  # lists read/written, rows materialised
    if not id_mask:
        assert c.young_seen_reads == 0 and c.young_seen_writes == 0


@pytest.mark.parametrize("list_cap,id_mask", [(4, 0x3FF), (12, 0), (16, 0)])
def test_young_seen_list_overflow(gossip, oracle, list_cap, id_mask):
    # lists that overflow -- in k_pull_young (more entries than it may keep) and in k_births (a
    # birth, or a whole id group, that does not fit): the node's young seen rows are materialised
    # and it dedups against dense seen words from then on (fresh tiles cleared at that node).
    # (C4's lists hold ~53 entries: none overflows at the default capacity)
    if list_cap == 16:  # 6,000 nodes, young tiles up to 5 hops: ~23 entries, k_pull_young keeps 8
        c = _parity(gossip, oracle, 6000, 16.0 / 5999, 83, 5.5, 5.0, dict(young_age=6, young_list_cap=list_cap),
                    flags=gossip.F_TILE_PER_TICK)
    elif list_cap == 12:  # (k_pull_young keeps 6 of them: ~11 entries per node here)
        c = _parity(gossip, oracle, 3000, 12.0 / 2999, 81, 6.0, 5.0, dict(young_age=4, young_list_cap=list_cap),
                    flags=gossip.F_TILE_PER_TICK)
    else:
        c = _parity(gossip, oracle, 400, 0.01, 73, 15.0, 5.0, dict(young_cap=8, young_age=4, young_list_cap=list_cap),
                    id_mask=id_mask, flags=gossip.F_TILE_PER_TICK)
    assert c.young_seen_reads > 0 and c.young_list_lines > 0  # some lists overflowed


@pytest.mark.parametrize("cap", [2, 127])
def test_young_collisions(gossip, oracle, cap):
    # 0x3FF id mask: id groups of several sources; group births resolve against slot arrivals
    _parity(gossip, oracle, 400, 0.01, 73, 15.0, 5.0, dict(young_cap=cap, young_age=4),
            id_mask=0x3FF, flags=gossip.F_TILE_PER_TICK)


def test_young_collisions_shared_tiles(gossip, oracle):
    # without a tile per tick: several ticks of births share one open tile
    _parity(gossip, oracle, 600, 0.008, 74, 12.0, 5.0, dict(young_cap=4, young_age=5), id_mask=0x7FF)


def test_young_odd_latency_cut(gossip, oracle):
    # a cut inside a tick (keep masks on young words) and a latency that does not divide 1 s
    _parity(gossip, oracle, 3000, 10.0 / 2999, 75, 7.37, 2.3, dict(young_cap=16, young_age=3),
            flags=gossip.F_TILE_PER_TICK)


def test_young_dense_graph(gossip, oracle):
    # p = 0.3: hundreds of peers per node (the gather walks several 64-peer chunks)
    _parity(gossip, oracle, 700, 0.3, 76, 5.6, 5.0, dict(young_cap=64, young_age=2),
            flags=gossip.F_TILE_PER_TICK)


def test_young_periodic_snapshots(gossip, oracle, monkeypatch):
    # PrintPeriodicStats partials counted inside k_pull_young (WF_SNAP) and k_births
    monkeypatch.setenv("GOSSIP_YOUNG", "1")
    monkeypatch.setenv("GOSSIP_YOUNG_CAP", "5")
    # (21 s: the snapshots at 10 s and 20 s, the second one inside the young-tile regime)
    sim = gossip.P2PGossipNetworkSimulation(1200, topo_seed=77, node_seed=78,
                                            flags=gossip.F_TILE_PER_TICK)
    sim.CreateRandomTopology(8.0 / 1199, 5.0)
    st = sim.Start(21.0)
    assert sim.engine.counters().young_launches > 0
    ref = oracle.run_reference(num_nodes=1200, connection_prob=8.0 / 1199, sim_time_s=21.0,
                               topo_seed=77, node_seed=78)
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(ref, k)), k
    got = [(gossip.seconds_to_ns(t), g, p, s) for t, g, p, s in sim.periodic]
    assert got == [tuple(x) for x in ref.periodic]


@pytest.mark.parametrize("case", ["overflow", "collisions", "odd_cut", "shared_tiles"])
def test_young_dense_rows(gossip, oracle, case):
    # dense-row tiles (pull_kernel.h) beside young tiles: k_pull_young writes every row of a tile
    # leaving the young set (YT_DW), k_pull reads it next tick without occupancy words -- with
    # overflowed slots, id-group births, an in-tick cut and tiles shared by several ticks
    dr = dict(dense_rows=1)
    if case == "overflow":
        c = _parity(gossip, oracle, 4096, 16.0 / 4095, 71, 6.0, 5.0, dict(dr, young_cap=1, young_age=3),
                    flags=gossip.F_TILE_PER_TICK)
        assert c.young_fallback_rows > 0 and c.pull_dense_tiles >= 0
    elif case == "collisions":
        _parity(gossip, oracle, 400, 0.01, 73, 15.0, 5.0, dict(dr, young_cap=2, young_age=4),
                id_mask=0x3FF, flags=gossip.F_TILE_PER_TICK)
    elif case == "odd_cut":
        _parity(gossip, oracle, 3000, 10.0 / 2999, 75, 7.37, 2.3, dict(dr, young_cap=16, young_age=3),
                flags=gossip.F_TILE_PER_TICK)
    else:
        _parity(gossip, oracle, 600, 0.008, 74, 12.0, 5.0, dict(dr, young_cap=4, young_age=5), id_mask=0x7FF)


def test_young_dense_rows_periodic_snapshots(gossip, oracle, monkeypatch):
    # periodic snapshot partials with dense-row tiles and saturation bits in play
    monkeypatch.setenv("GOSSIP_YOUNG", "1")
    monkeypatch.setenv("GOSSIP_DENSE_ROWS", "1")
    sim = gossip.P2PGossipNetworkSimulation(1200, topo_seed=77, node_seed=78, flags=gossip.F_TILE_PER_TICK)
    sim.CreateRandomTopology(8.0 / 1199, 5.0)
    st = sim.Start(21.0)
    c = sim.engine.counters()
    assert c.young_launches > 0 and c.pull_sat == 1
    ref = oracle.run_reference(num_nodes=1200, connection_prob=8.0 / 1199, sim_time_s=21.0,
                               topo_seed=77, node_seed=78)
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(ref, k)), k
    got = [(gossip.seconds_to_ns(t), g, p, s) for t, g, p, s in sim.periodic]
    assert got == [tuple(x) for x in ref.periodic]


@pytest.mark.parametrize("overlap,nt", [(0, 1), (1, 1), (1, 0)])
def test_young_off_equals_on(gossip, overlap, nt):
    # 200k nodes (below the auto threshold): forced on == forced off, collisions included, with
    # k_pull_young after k_pull (0) or concurrent on a second stream (1), its slot lines read
    # non-temporally (young_nt 1, the default) or cached
    n = 200_000
    topo = gossip.Topology.gnp(n, 16.0 / (n - 1), 79, gossip.TOPO_SKIP, threads=16)
    t_cut = gossip.seconds_to_ns(5.2)
    ev = gossip.make_schedule(n, 80, T0, t_cut, id_mask=0xFFFFF)
    lat = gossip.milliseconds_to_ns(5.0)
    on = _run(gossip, topo, ev, lat, t_cut, dict(young=1, young_overlap=overlap, young_nt=nt), flags=gossip.F_TIMING)
    off = _run(gossip, topo, ev, lat, t_cut, dict(young=0))
    a, b = on.stats(), off.stats()
    c = on.counters()
    assert c.young_launches > 0 and off.counters().young_launches == 0
    assert c.pull_phase_ms > 0
    for k in STATS:
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    on.close()
    off.close()


# Empty-slot skipping (round 6, option young_skip, young_kernel.h): writers of non-empty slots stamp
# their peers' hint bytes, and the next tick's readers load only stamped peers' slot lines.  Forced on
# every tick (1) it must still equal the oracle through overflowed slots (cap 1: headers read through
# the stamp), two-line slots (cap 64 on a dense graph, > 64 peers per node), k_births' first entries
# (a birth into an empty slot stamps it) and id groups; 0 turns it off; auto (-1) fires on the sparse
# ticks of these small graphs (births and their first hop).
@pytest.mark.parametrize("case", ["overflow", "groups", "dense", "shared", "off", "auto"])
def test_young_empty_slot_skipping(gossip, oracle, case):
    tpt = gossip.F_TILE_PER_TICK
    if case == "overflow":
        c = _parity(gossip, oracle, 4096, 16.0 / 4095, 71, 6.0, 5.0, dict(young_cap=1, young_age=3, young_skip=1), flags=tpt)
        assert c.young_fallback_rows > 0
    elif case == "groups":
        c = _parity(gossip, oracle, 400, 0.01, 73, 15.0, 5.0, dict(young_cap=2, young_age=4, young_skip=1),
                    id_mask=0x3FF, flags=tpt)
    elif case == "dense":
        c = _parity(gossip, oracle, 700, 0.3, 76, 5.6, 5.0, dict(young_cap=64, young_age=2, young_skip=1), flags=tpt)
    elif case == "shared":
        c = _parity(gossip, oracle, 600, 0.008, 74, 12.0, 5.0, dict(young_cap=4, young_age=5, young_skip=1), id_mask=0x7FF)
    elif case == "off":
        c = _parity(gossip, oracle, 4096, 16.0 / 4095, 71, 6.0, 5.0, dict(young_age=5, young_skip=0), flags=tpt)
        assert c.young_skip_ticks == 0
        return
    else:
        c = _parity(gossip, oracle, 4096, 16.0 / 4095, 71, 6.0, 5.0, dict(young_age=5, young_skip=-1), flags=tpt)
        assert 0 < c.young_skip_ticks < c.young_launches
        return
    assert c.young_skip_ticks > 0 and c.young_launches > 0


# The idle-node pass (round 6, option young_idle, k_young_idle): on a tick whose k_pull_young reads
# only stamped slots and keeps every seen list, nodes without a stamped peer skip the node walk --
# an empty slot and the list header's kept part written by the pass instead.  With id groups (births
# testing their group against the list's kept entries), overflowing lists (fresh tiles cleared by the
# walk) and young tiles of every age, on and off must both equal the oracle.
@pytest.mark.parametrize("case", ["plain", "groups", "list_overflow", "off"])
def test_young_idle_nodes(gossip, oracle, case):
    tpt = gossip.F_TILE_PER_TICK
    if case == "plain":
        c = _parity(gossip, oracle, 4096, 16.0 / 4095, 71, 6.0, 5.0, dict(young_age=5, young_skip=1), flags=tpt)
    elif case == "groups":
        c = _parity(gossip, oracle, 400, 0.01, 73, 15.0, 5.0, dict(young_cap=3, young_age=5, young_skip=1),
                    id_mask=0x3FF, flags=tpt)
    elif case == "list_overflow":
        c = _parity(gossip, oracle, 400, 0.01, 73, 15.0, 5.0, dict(young_cap=8, young_age=4, young_list_cap=4, young_skip=1),
                    id_mask=0x3FF, flags=tpt)
    else:
        c = _parity(gossip, oracle, 4096, 16.0 / 4095, 71, 6.0, 5.0, dict(young_age=5, young_skip=1, young_idle=0), flags=tpt)
        assert c.young_idle_ticks == 0
        return
    assert c.young_idle_ticks > 0
