"""The BASELINE.json configurations themselves under test on the GPU (C2, C4, C5), not just
smaller stand-ins.

C4 (10M nodes): a bounded sample replayed against ORACLE A bit for bit -- real generations of
the bench's slice plus id groups built on the C4 graph (the id-collision paths of p2pnode.cc:189
at full size) -- through every pull variant the bench can select (non-temporal rows, the 16,384-
block grid, a grid of 3 blocks that makes every wave stride over thousands of chunks) and as two
share shards; then the bench's own steady-state slice (shard 0 of 2, ~280 GiB) against the
invariants of the reference's counters.
C5 (65,536 nodes, p = 0.3, 4,096 concurrent shares): MFMA == CSR pull, a 64-share subset ==
ORACLE B, row partitions of 2 and 8 ranks == the single engine.
C2 (4,096 nodes, p = 0.3, full 60 s): MFMA tick-by-tick, MFMA hop-batched and the CSR pull ==
ORACLE B over all ~64k shares.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STATS = ("gen", "recv", "fwd", "sent", "processed", "peers", "sockets")
SUM_STATS = ("gen", "recv", "fwd", "sent", "processed")


def _w():
    import gossip.workloads as W
    return W


def _same(st, ref, keys=STATS, what=""):
    for k in keys:
        a, b = getattr(st, k), getattr(ref, k)
        assert np.array_equal(a, b), (what, k, int(np.count_nonzero(a != b)))


def _run(gossip, topo, ev, t_start, t_cut, options=(), close=True, **kw):
    eng = gossip.Engine(topo.num_nodes, _w().L_NS, t_start, t_cut, **kw)
    for k, v in options:
        eng.set_option(k, v)
    eng.set_topology(topo)
    eng.set_schedule(ev)
    eng.run()
    eng.sync()
    st, c = eng.stats(), eng.counters()
    if close:
        eng.close()
        return st, c
    return st, c, eng


def _sum(stats):
    out = {}
    for k in SUM_STATS:
        out[k] = sum(getattr(s, k).astype(np.uint64) for s in stats)
    return out


def _invariants(st, c=None):
    assert np.array_equal(st.fwd, st.recv)  # p2pnode.cc:157,163
    assert np.array_equal(st.sent, st.peers.astype(np.uint64) * (st.gen + st.recv).astype(np.uint64))
    assert np.all(st.processed <= st.gen + st.recv)
    if c is not None:
        assert c.edge_events == int(st.sent.sum())


# ------------------------------------------------------------------------------------------- C4
@pytest.fixture(scope="module")
def c4(gossip):
    W = _w()
    topo = W.topology("C4")
    rp, col, _ = topo.csr()
    return topo, rp, col


def _ring(rp, col, src, d):
    """Nodes at exact BFS distance d from src (d small: the levels stay tiny)."""
    seen = {int(src)}
    level = [int(src)]
    for _ in range(d):
        nxt = []
        for u in level:
            for v in col[rp[u]:rp[u + 1]].tolist():
                if v not in seen:
                    seen.add(v)
                    nxt.append(v)
        level = nxt
    return sorted(level)


def _c4_sample(gossip, c4):
    """Six real generations of the bench slice + five id groups placed on the C4 graph."""
    W = _w()
    topo, rp, col = c4
    n = topo.num_nodes
    L, T = W.L_NS, W.SLICE_NS
    ev = gossip.make_schedule(n, W.CONFIGS["C4"]["node_seed"], W.T0_NS, W.T_CUT_NS,
                              t_gen_end_ns=T + L, threads=16)
    base = ev[ev["ns"] >= T][:6]
    used = set(base["node"].tolist())
    rows = []
    gid = 0xC4C40000

    def pick(cands):
        for v in cands:
            if v not in used:
                used.add(v)
                return v
        raise AssertionError("no free node")

    # deterministic anchors far apart in id space
    anchors = [1_234_567, 3_456_789, 5_678_901, 7_890_123, 9_012_345]
    t1 = T + L + 200_000  # tick 2001, phase 0.2 ms
    # G1: the flood reaches b (distance 2) first, b generates 1 us later: gen + sent count,
    #     processed does not (p2pnode.cc:115-120 with the id already in processedShares)
    a = pick([anchors[0]]); b = pick(_ring(rp, col, a, 2))
    rows += [(t1, a, gid), (t1 + 2 * L + 1000, b, gid)]
    # G2: b generates 1 us BEFORE the flood's arrival in the same tick: the arrival is dropped
    a = pick([anchors[1]]); b = pick(_ring(rp, col, a, 2))
    rows += [(t1, a, gid + 1), (t1 + 2 * L - 1000, b, gid + 1)]
    # G3: two floods of one id meet in the middle (distance 4, phases 500 ns apart)
    a = pick([anchors[2]]); b = pick(_ring(rp, col, a, 4))
    rows += [(t1, a, gid + 2), (t1 + 500, b, gid + 2)]
    # G4: three sources in one tick, pairwise >= 2 hops apart, phases in reverse node order
    a = pick([anchors[3]]); b = pick(_ring(rp, col, a, 2)); c = pick(_ring(rp, col, a, 3))
    rows += [(t1 + 300_000, a, gid + 3), (t1 + 200_000, b, gid + 3), (t1 + 100_000, c, gid + 3)]
    # G5: a tie -- b (a peer of a) generates at the very ns a's share arrives: the generation
    #     event was scheduled first and wins
    a = pick([anchors[4]]); b = pick(_ring(rp, col, a, 1))
    rows += [(t1, a, gid + 4), (t1 + L, b, gid + 4)]
    r = np.array(rows, dtype=np.int64)
    grp = gossip.events_from_arrays(r[:, 0], r[:, 1], r[:, 2])
    out = np.concatenate([base, grp])
    out = out[np.lexsort((out["node"], out["ns"]))]
    assert len(np.unique(base["share_id"])) == len(base) and not np.isin(grp["share_id"], base["share_id"]).any()
    # PrintStatistics half-way through tick 2005: the base shares (tick 2000) count 5 hops, the
    # groups (tick 2001) 4 hops if their phase is below L/2, else 3
    return out, T + 5 * L + L // 2


def test_c4_sample_matches_oracle_a(gossip, oracle, c4):
    from concurrent.futures import ThreadPoolExecutor

    W = _w()
    topo = c4[0]
    n = topo.num_nodes
    ev, t_cut = _c4_sample(gossip, c4)
    a, b = topo.links()
    # ORACLE A (CPU, ~30 s at 10M nodes; the ctypes call releases the GIL) runs beside the GPU
    # variants below
    pool = ThreadPoolExecutor(1)
    fut = pool.submit(oracle.run_replay, n, W.L_NS, W.T0_NS, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"])
    # (the sample's window is <= 16 words: the pull is k_pull<8..16, 1>, whatever pull_lpw says;
    # young_overlap 0 and pull_gate 0 are test_young_gpu's and test_late_exit_gpu's)
    variants = [
        ("auto (this 11-generation sample is too thin for young tiles)", ()),
        ("young-tile slots forced on", (("young", 1),)),
        ("young tiles, 8-entry slots (overflow paths at scale)", (("young", 1), ("young_cap", 8))),
        ("nt rows, 16384-block grid (k_pull<8..16,1,false>: this sample's window is <= 16 words; "
         "the production k_pull<32,1,true> is test_c4_headline_kernels_match_oracle_b's)", (("pull_nt", 1), ("pull_grid", 16384))),
        ("nt rows, 3-block grid", (("pull_nt", 1), ("pull_grid", 3))),
        ("no bottom-up early exit (late_age 0; the default exits on every tile)", (("late_age", 0),)),
    ]
    runs = []
    for name, opts in variants:
        runs.append((name, opts) + _run(gossip, topo, ev, W.T0_NS, t_cut, options=opts, max_words=16))
    ref = fut.result()
    pool.shutdown()
    del a, b
    assert ref.edge_events > 10_000_000 and int((ref.gen + ref.recv - ref.processed).sum()) >= 1
    for name, opts, st, c in runs:
        _same(st, ref, what=name)
        if opts and opts[0] == ("pull_nt", 1):
            assert c.pull_nt == 1 and c.pull_grid == dict(opts)["pull_grid"]
    parts = [_run(gossip, topo, ev, W.T0_NS, t_cut, max_words=16, shard_rank=r, shard_count=2)[0]
             for r in range(2)]
    tot = _sum(parts)
    for k in SUM_STATS:
        assert np.array_equal(tot[k], getattr(ref, k).astype(np.uint64)), ("2 shards", k)
    # the 8-GPU layout's rule (bench.shard_flags): 8 shards by birth tick, a fresh tile per birth
    # tick -- an id instance stays whole on the shard of its first generation (G1-G5 above: later
    # generations of an instance in its old tile) -- with young tiles, empty-slot skipping and the
    # idle-node pass forced (the sample is too thin for their auto rules)
    tick = gossip.F_SHARD_BY_TICK | gossip.F_TILE_PER_TICK
    own = gossip.shard_events(topo, ev, 8, by_tick_latency_ns=W.L_NS)
    busy = sorted(set(own.tolist()))  # (the other shards own no event: all-zero counters)
    assert len(busy) >= 2
    for opts in ((), (("young", 1), ("young_skip", 1), ("young_cap", 8))):
        runs8 = [_run(gossip, topo, ev, W.T0_NS, t_cut, options=opts, max_words=16, shard_rank=r, shard_count=8,
                      flags=tick) for r in busy]
        tot = _sum([st for st, _ in runs8])
        for k in SUM_STATS:
            assert np.array_equal(tot[k], getattr(ref, k).astype(np.uint64)), ("8 shards by birth tick", opts, k)
        assert sum(c.edge_events for _, c in runs8) == ref.edge_events
        if opts:
            assert sum(c.young_skip_ticks for _, c in runs8) > 0 and sum(c.young_idle_ticks for _, c in runs8) > 0


def _c4_headline_sample(gossip, c4, per_tick=20, ticks=24):
    """Distinct-id generations of the bench's slice: `per_tick` of every tick of [2000, 2000 +
    ticks), evenly spaced in the tick's (ns, node) order; floods cut ~6 hops after the last tick."""
    W = _w()
    n = c4[0].num_nodes
    L, T = W.L_NS, W.SLICE_NS
    ev, _ = W.slice_schedule(n, W.CONFIGS["C4"]["node_seed"], T, T + ticks * L)
    win = ev[ev["ns"] >= T]
    # ids that occur once in the slice (ORACLE B covers distinct ids only)
    ids, cnt = np.unique(ev["share_id"], return_counts=True)
    win = win[np.isin(win["share_id"], ids[cnt == 1])]
    tick = win["ns"] // L
    pick = []
    for k in range(T // L, T // L + ticks):
        idx = np.flatnonzero(tick == k)
        pick.append(idx[np.linspace(0, len(idx) - 1, per_tick).astype(np.int64)])
    out = np.ascontiguousarray(win[np.concatenate(pick)])
    assert len(np.unique(out["share_id"])) == len(out) == per_tick * ticks
    return out, T + (ticks + 6) * L + L // 2


def test_c4_headline_kernels_match_oracle_b(gossip, oracle, c4):
    # The kernels that produce the bench's number, in the bench's configuration: k_pull<32,1,true>
    # (windows > 64 words: 32 word-lanes per node, non-temporal rows, tile lists in age order, the
    # 16,384-block grid, the early exit on every tile, saturation bits, dense-row tiles) beside
    # k_pull_young (young_nt slot reads, concurrent on the second stream) -- on the C4 graph against
    # ORACLE B (p2pnode.cc:127-199).  A fresh tile per tick (F_TILE_PER_TICK) gives the window of ~25
    # tiles those kernels need at a CPU-checkable 480 generations; young tiles and NT rows are forced
    # (auto keys them off the slice's full ~14k births per tick); dense rows are forced on every
    # listed tile (auto: a 20-share tile's rows are not dense).
    W = _w()
    topo = c4[0]
    n = topo.num_nodes
    ev, t_cut = _c4_headline_sample(gossip, c4)
    a, b = topo.links()
    ref = oracle.run_oracle_b(n, W.L_NS, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"], threads=16)
    del a, b
    assert ref.edge_events > 1e10
    prod = (("young", 1), ("young_nt", 1), ("pull_nt", 1), ("pull_grid", 16384), ("pull_tile_order", 1))
    # (saturation bits and dense rows off: tests/test_engine_gpu.py's option variants, small graphs)
    variants = [
        ("production kernels, dense rows auto", prod),
        ("production kernels, dense rows on every listed tile", prod + (("dense_rows", 1),)),
    ]
    for name, opts in variants:
        st, c = _run(gossip, topo, ev, W.T0_NS, t_cut, options=opts, flags=gossip.F_TILE_PER_TICK)
        _same(st, ref, what=name)
        assert c.edge_events == ref.edge_events, name
        # the instantiation: k_pull<32, 1, true> over tile lists, early exit on, k_pull_young ran
        assert c.words_hw > 64 and c.pull_lpw == 32 and c.pull_nt == 1 and c.pull_grid == 16384, name
        assert c.pull_tiles == 1 and c.pull_late_age == 1 and c.young_launches > 0, name
        if dict(opts).get("pull_sat", 1):
            assert c.pull_sat == 1 and c.pull_sat_skips > 0, name
    # the same kernels as the 8 ranks of the 8-GPU layout run them (bench.shard_flags: birth-tick
    # rule, a fresh tile per birth tick), every sparse-tick path forced: empty-slot skipping and the
    # idle-node pass in k_pull_young, push marks in k_pull and k_births (pull_push 1: every listed
    # tile; a shard's window here is <= 3 tiles, so its k_pull is the narrow one -- the production
    # k_pull<32,1,..,PUSH> at C4 scale is test_c4_tick_rule_slice_equals_continuous_run's)
    # Two of the eight shards, each against ORACLE B on its own generations (a shard is a whole
    # job of its share instances: its counters are the reference's for those shares alone)
    tick = gossip.F_SHARD_BY_TICK | gossip.F_TILE_PER_TICK
    sparse = prod + (("young_skip", 1), ("pull_push", 1))
    own = gossip.shard_events(topo, ev, 8, by_tick_latency_ns=W.L_NS)
    a, b = topo.links()
    for r in (1, 6):
        mine = ev[own == r]
        ref_r = oracle.run_oracle_b(n, W.L_NS, t_cut, a, b, mine["ns"], mine["node"], mine["share_id"], threads=16)
        st, c = _run(gossip, topo, ev, W.T0_NS, t_cut, options=sparse, flags=tick, shard_rank=r, shard_count=8)
        _same(st, ref_r, keys=SUM_STATS, what=f"shard {r} of 8 by birth tick")
        assert c.edge_events == ref_r.edge_events and c.young_skip_ticks > 0 and c.young_idle_ticks > 0, r
    del a, b


def _c4_shard_deltas(gossip, topo, ev, shard, shards, t0, t1, options=(), flags=0):
    W = _w()
    eng = gossip.Engine(topo.num_nodes, W.L_NS, W.T0_NS, W.T_CUT_NS, shard_rank=shard, shard_count=shards,
                        flags=flags)
    for k, v in options:
        eng.set_option(k, v)
    eng.set_topology(topo)
    eng.set_schedule(ev)
    eng.run(t0)
    eng.sync()
    s0, c0 = eng.stats(), eng.counters()
    eng.run(t1)
    eng.sync()
    s1, c1 = eng.stats(), eng.counters()
    eng.close()
    return s0, s1, c0, c1


def test_c4_bench_slice_equals_continuous_run(gossip, c4):
    # The bench's workload is the warm-start slice (every generation of the 16 ticks before
    # t = 10 s and of the timed ticks, plus all earlier generations of their ids), ramped, then
    # timed over ticks [2005, 2025).  Pinned here against the CONTINUOUS run (every generation
    # from t = 5 s) of the same share shard: the per-node recv deltas and the edge events of the
    # timed ticks must be identical (p2pnode.cc:189: an id's earlier floods are in the seen-sets
    # either way).  Shard 0 of 8 (the 8-GPU layout's share shard): the continuous run's start-up
    # (the renewal density peaks ~7 s) needs ~25 % more live words than the steady state, and
    # the eighth keeps the 1,000 ticks from t = 5 s short.
    W = _w()
    topo = c4[0]
    n = topo.num_nodes
    warm, steps = 5, 20
    t0 = W.SLICE_NS // W.L_NS + warm
    t1 = t0 + steps
    ev_s, info = W.slice_schedule(n, W.CONFIGS["C4"]["node_seed"], W.SLICE_NS, t1 * W.L_NS)
    assert info["earlier_same_id"] > 0
    ev_c = gossip.make_schedule(n, W.CONFIGS["C4"]["node_seed"], W.T0_NS, W.T_CUT_NS, t_gen_end_ns=t1 * W.L_NS,
                                threads=16)
    shards = 16  # (the hash rule's eighth is test_c4_tick_rule_...'s layout now: a sixteenth keeps this short)
    own_s, own_c = gossip.shard_events(topo, ev_s, shards), gossip.shard_events(topo, ev_c, shards)
    # the slice's events are a subset of the continuous run's, each on the same shard
    key = lambda e: (e["ns"].astype(np.int64) << 24) | e["node"].astype(np.int64)  # noqa: E731 (ns < 2^34, n < 2^24)
    sl_in_c = np.isin(key(ev_c), key(ev_s))
    assert int(sl_in_c.sum()) == len(ev_s)
    assert np.array_equal(own_c[sl_in_c], own_s)
    # young tiles forced on: auto turns them off at 8 shards (~12 slot entries per node, §3), the
    # 2-shard bench runs them
    yo = (("young", 1),)
    a0, a1, ca0, ca1 = _c4_shard_deltas(gossip, topo, ev_s, 0, shards, t0, t1, yo)
    b0, b1, cb0, cb1 = _c4_shard_deltas(gossip, topo, ev_c, 0, shards, t0, t1, yo)
    for k in ("recv", "gen", "sent", "processed"):
        da = getattr(a1, k).astype(np.int64) - getattr(a0, k).astype(np.int64)
        db = getattr(b1, k).astype(np.int64) - getattr(b0, k).astype(np.int64)
        assert np.array_equal(da, db), (k, int(np.count_nonzero(da != db)))
    assert ca1.edge_events - ca0.edge_events == cb1.edge_events - cb0.edge_events > 0
    # the slice run itself against the reference's counter invariants
    _invariants(a1, ca1)
    mine = ev_s[own_s == 0]
    gens = mine[mine["ns"] < t1 * W.L_NS]
    assert int(a1.gen.sum()) == len(gens) == ca1.generations
    assert np.array_equal(a1.gen, np.bincount(gens["node"], minlength=n).astype(np.uint32))
    # later generations of ids whose earlier flood already covered the node: counted, not processed
    assert int((a1.gen.astype(np.int64) + a1.recv - a1.processed).sum()) > 0
    assert ca1.words_hw > 100 and int(a1.recv.sum()) > 100 * len(gens)  # (a sixteenth: ~160 words)
    # the bench's pull: young-tile slots, the early exit on every tile
    assert ca1.young_launches > 0 and ca1.pull_late_age == 1


def test_c4_tick_rule_slice_equals_continuous_run(gossip, c4):
    # The 8-GPU layout's own rank (bench.shard_flags at 8 shards: birth-tick rule, a fresh tile per
    # birth tick, young tiles and every sparse-tick path on auto -- empty-slot skipping, the
    # idle-node pass, push marks in the production k_pull<32,1,true,SP,PUSH>): shard 1 of 8 of the
    # bench's warm-start slice against the continuous run from t = 5 s of the same shard, per-node
    # deltas of the timed ticks bit-identical (the slice is exact iff every older flood has died out,
    # DESIGN.md section 4), and both against the reference's counter invariants.
    W = _w()
    topo = c4[0]
    n = topo.num_nodes
    warm, steps = 5, 20
    t0 = W.SLICE_NS // W.L_NS + warm
    t1 = t0 + steps
    ev_s, _ = W.slice_schedule(n, W.CONFIGS["C4"]["node_seed"], W.SLICE_NS, t1 * W.L_NS)
    ev_c = gossip.make_schedule(n, W.CONFIGS["C4"]["node_seed"], W.T0_NS, W.T_CUT_NS, t_gen_end_ns=t1 * W.L_NS,
                                threads=16)
    shards, shard = 8, 1
    own_s = gossip.shard_events(topo, ev_s, shards, by_tick_latency_ns=W.L_NS)
    tick = gossip.F_SHARD_BY_TICK | gossip.F_TILE_PER_TICK
    a0, a1, ca0, ca1 = _c4_shard_deltas(gossip, topo, ev_s, shard, shards, t0, t1, flags=tick)
    b0, b1, cb0, cb1 = _c4_shard_deltas(gossip, topo, ev_c, shard, shards, t0, t1, flags=tick)
    for k in ("recv", "gen", "sent", "processed"):
        da = getattr(a1, k).astype(np.int64) - getattr(a0, k).astype(np.int64)
        db = getattr(b1, k).astype(np.int64) - getattr(b0, k).astype(np.int64)
        assert np.array_equal(da, db), (k, int(np.count_nonzero(da != db)))
    assert ca1.edge_events - ca0.edge_events == cb1.edge_events - cb0.edge_events > 0
    _invariants(a1, ca1)
    _invariants(b1, cb1)
    mine = ev_s[own_s == shard]
    gens = mine[mine["ns"] < t1 * W.L_NS]
    assert int(a1.gen.sum()) == len(gens) == ca1.generations
    # the sparse-tick paths ran in the timed ticks (counters restart at reset_timing: c1 - c0 here
    # is cumulative since creation, so check the slice run's totals)
    assert ca1.young_skip_ticks > 0 and ca1.young_idle_ticks > 0, "empty-slot skipping / idle pass"
    assert ca1.pull_push_tiles > 0 and ca1.pull_marks > 0 and ca1.pull_lpw == 32, "push marks"


# ------------------------------------------------------------------------------------------- C5
@pytest.fixture(scope="module")
def c5(gossip):
    W = _w()
    return W.topology("C5"), W.c5_flood()


def test_c5_mfma_equals_csr_and_oracle_b(gossip, oracle, c5):
    W = _w()
    topo, ev = c5
    n = topo.num_nodes
    t_cut = W.T0_NS + 40 * W.L_NS
    dense, cd = _run(gossip, topo, ev, W.T0_NS, t_cut, mode=gossip.MODE_DENSE)
    assert cd.dense_fused_launches == cd.pull_launches
    csr, _ = _run(gossip, topo, ev, W.T0_NS, t_cut, mode=gossip.MODE_CSR)
    _same(dense, csr, what="C5 MFMA vs CSR, 4096 shares")
    three, _ = _run(gossip, topo, ev, W.T0_NS, t_cut, mode=gossip.MODE_DENSE, options=(("dense_fused", 0),))
    _same(dense, three, what="C5 fused vs three-kernel MFMA, 4096 shares")
    _invariants(dense, cd)
    assert cd.dense_ops > 0 and int(dense.recv.sum()) == len(ev) * (n - 1)  # diameter 2: all reached
    sub = ev[:64]
    a, b = topo.links()
    ref = oracle.run_oracle_b(n, W.L_NS, t_cut, a, b, sub["ns"], sub["node"], sub["share_id"], threads=16)
    del a, b
    for mode in (gossip.MODE_DENSE, gossip.MODE_CSR):
        st, _ = _run(gossip, topo, sub, W.T0_NS, t_cut, mode=mode)
        _same(st, ref, what=f"C5 64 shares mode {mode} vs ORACLE B")


@pytest.mark.parametrize("ranks", [8])  # (2 ranks: tests/test_multiprocess_gpu.py, test_row_partition.py)
def test_c5_row_partition_sums_to_single(gossip, c5, ranks):
    W = _w()
    topo, ev = c5
    t_cut = W.T0_NS + 40 * W.L_NS
    whole, _ = _run(gossip, topo, ev, W.T0_NS, t_cut, mode=gossip.MODE_DENSE)
    engs = []
    for r in range(ranks):
        e = gossip.Engine(topo.num_nodes, W.L_NS, W.T0_NS, t_cut, mode=gossip.MODE_DENSE)
        e.set_row_partition(r, ranks)
        e.set_topology(topo)
        e.set_schedule(ev)
        engs.append(e)
    gossip.group_run(engs)
    parts = [e.stats() for e in engs]
    cs = [e.counters() for e in engs]
    for e in engs:
        e.close()
    tot = _sum(parts)
    for k in SUM_STATS:
        assert np.array_equal(tot[k], getattr(whole, k).astype(np.uint64)), (ranks, k)
    # every rank's every tick ran k_dense_fused over its own rows (round 6) and the ranks exchanged
    # FT slices: per tick, each rank sends its rows' bits of every window column
    for c in cs:
        assert c.dense_fused_launches == c.pull_launches > 0, (c.dense_fused_launches, c.pull_launches)
        assert c.exchange_bytes_sent >= c.pull_launches * 4096 * (topo.num_nodes // ranks) // 8


# ------------------------------------------------------------------------------------------- C2
def test_c2_full_run_all_paths_match_oracle_b(gossip, oracle):
    W = _w()
    cfg = W.CONFIGS["C2"]
    topo = W.topology("C2")
    n = topo.num_nodes
    ev = gossip.make_schedule(n, cfg["node_seed"], W.T0_NS, W.T_CUT_NS, threads=16)
    a, b = topo.links()
    ref = oracle.run_oracle_b(n, W.L_NS, W.T_CUT_NS, a, b, ev["ns"], ev["node"], ev["share_id"], threads=16)
    assert ref.edge_events > 1e11
    runs = [("MFMA tick-by-tick", dict(mode=gossip.MODE_DENSE)),
            ("MFMA hop-batched", dict(mode=gossip.MODE_DENSE, flags=gossip.F_HOP_BATCH)),
            ("MFMA hop-batched, three kernels", dict(mode=gossip.MODE_DENSE, flags=gossip.F_HOP_BATCH,
                                                     options=(("dense_fused", 0),))),
            ("CSR hop-batched", dict(mode=gossip.MODE_CSR, flags=gossip.F_HOP_BATCH)),
            ("AUTO", dict())]
    for name, kw in runs:
        st, c = _run(gossip, topo, ev, W.T0_NS, W.T_CUT_NS, **kw)
        _same(st, ref, what=name)
        assert c.edge_events == ref.edge_events
        if name == "AUTO":
            assert c.dense_ops > 0  # AUTO picks the MFMA path on a p = 0.3 graph
        if name.startswith("MFMA"):  # every MFMA tick fused (unique ids) unless switched off
            assert c.dense_fused_launches == (0 if "three" in name else c.pull_launches), name


def test_c2_golden_fixture_on_every_path(gossip):
    # tests/golden/n4096_p03_short (C2's graph shape, ORACLE A output): the MFMA contraction tick
    # by tick and hop-batched, and the CSR pull, each bit-exact against the fixture
    import golden_util as G
    W = _w()
    g = G.load("n4096_p03_short")
    p = g["params"]
    n = p["num_nodes"]
    topo = gossip.Topology.gnp(n, p["connection_prob"], p["topo_seed"], gossip.TOPO_EXACT)
    lat = gossip.milliseconds_to_ns(p["latency_ms"])
    t_cut = gossip.seconds_to_ns(p["sim_time_s"] - 0.1)
    ev = gossip.make_schedule(n, p["node_seed"], W.T0_NS, t_cut)
    for kw in (dict(mode=gossip.MODE_DENSE), dict(mode=gossip.MODE_DENSE, flags=gossip.F_HOP_BATCH),
               dict(mode=gossip.MODE_CSR), dict(mode=gossip.MODE_AUTO)):
        eng = gossip.Engine(n, lat, W.T0_NS, t_cut, **kw)
        eng.set_topology(topo)
        eng.set_schedule(ev)
        eng.run()
        st = eng.stats()
        if kw["mode"] == gossip.MODE_AUTO:
            assert eng.mode == gossip.MODE_DENSE
        eng.close()
        for k in G.STAT_KEYS:
            assert np.array_equal(getattr(st, k), g[k]), (kw, k)
