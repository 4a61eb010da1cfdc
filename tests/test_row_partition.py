"""Row partition: engine r of R pulls, dedups and counts only its block of node
rows and the ranks exchange frontier rows, tile occupancy and liveness after every tick, in
`xchunks` row chunks (the pipelined exchange).  The lockstep one-device backend
(gossip_engine_group_run) must give per-node counters that sum to the single engine's and to
ORACLE A's bit for bit; the RCCL backend is exercised on one rank (ncclBroadcast / all-gather
over a 1-rank communicator)."""
import numpy as np
import pytest

from cases import L, T0

pytestmark = pytest.mark.gpu

SUM = ("gen", "recv", "fwd", "sent", "processed")


def _inputs(gossip, n, p, seed, t_cut_s):
    topo = gossip.Topology.gnp(n, p, seed, gossip.TOPO_EXACT)
    t_cut = gossip.seconds_to_ns(t_cut_s)
    ev = gossip.make_schedule(n, seed + 1, T0, t_cut)
    return topo, t_cut, ev


def _engine(gossip, n, t_cut, topo, ev, mode, flags, part=None, snaps=()):
    e = gossip.Engine(n, L, T0, t_cut, mode=mode, flags=flags)
    if part:
        e.set_row_partition(*part)
    e.set_topology(topo)
    for t in snaps:
        e.add_snapshot(t)
    e.set_schedule(ev)
    return e


# dense ranks run the fused tick (k_dense_fused over their own rows, FT slices exchanged: round 6)
# unless "dense3" (dense_fused 0: the three-kernel pull and the chunked F-row exchange)
@pytest.mark.parametrize("mode,n,p,R,batch,xchunks", [
    ("csr", 1500, 0.01, 2, False, 4),
    ("csr", 1500, 0.01, 3, False, 1),
    ("dense", 1200, 0.3, 2, False, 4),
    ("dense3", 1200, 0.3, 2, False, 4),
    ("csr", 1100, 0.02, 2, True, 2),
    ("dense", 1100, 0.3, 2, True, 1),
    ("csr", 5000, 0.004, 2, False, 3),   # chunks of 1,024 rows, none empty
    ("dense", 1500, 0.3, 3, False, 16),  # ranks of 512, 512, 476 rows: 1,024-node stage 0 spans two
    ("dense3", 2100, 0.3, 2, False, 16),  # many empty chunks
])
def test_group_run_matches_single_engine_and_oracle(gossip, oracle, mode, n, p, R, batch, xchunks):
    topo, t_cut, ev = _inputs(gossip, n, p, 31, 7.3)
    m = gossip.MODE_DENSE if mode.startswith("dense") else gossip.MODE_CSR
    flags = gossip.F_HOP_BATCH if batch else 0
    snaps = [gossip.seconds_to_ns(6.0), gossip.seconds_to_ns(7.0)]
    ref = _engine(gossip, n, t_cut, topo, ev, m, flags, snaps=snaps)
    ref.run()
    ref.sync()
    want = ref.stats()
    want_snap = [ref.snapshot(k) for k in range(len(snaps))]
    ranks = [_engine(gossip, n, t_cut, topo, ev, m, flags, part=(r, R), snaps=snaps) for r in range(R)]
    for e in ranks:  # pipelined exchange: rows pulled and exchanged in xchunks row chunks
        e.set_option("xchunks", xchunks)
        if mode == "dense3":
            e.set_option("dense_fused", 0)
    gossip.group_run(ranks)
    for e in ranks:
        e.sync()
    got = [e.stats() for e in ranks]
    for e in ranks:  # every dense tick of every rank fused (unique ids), or none
        c = e.counters()
        if mode == "dense":
            assert c.dense_fused_launches == c.pull_launches > 0 and c.exchange_bytes_sent > 0
        elif mode == "dense3":
            assert c.dense_fused_launches == 0
    for k in SUM:
        total = sum(getattr(g, k).astype(np.uint64) for g in got)
        assert np.array_equal(total, getattr(want, k).astype(np.uint64)), k
    for k in ("peers", "sockets"):
        assert np.array_equal(getattr(got[0], k), getattr(want, k)), k
    # each rank counts only its own rows
    owned = [np.nonzero(g.recv)[0] for g in got]
    for r in range(R - 1):
        assert owned[r].size == 0 or owned[r + 1].size == 0 or owned[r].max() < owned[r + 1].min()
    for k, (t_ns, g_tot, p_tot) in enumerate(want_snap):
        parts = [e.snapshot(k) for e in ranks]
        assert all(x[0] == t_ns and x[1] == g_tot for x in parts)
        assert sum(x[2] for x in parts) == p_tot
    # ORACLE A on the sparse cases (seconds); the dense single engine is pinned to ORACLE A in
    # test_engine_gpu.py (here its event loop would take ~30 s per case)
    if n <= 1500 and mode == "csr":
        a, b = topo.links()
        r = oracle.run_replay(n, L, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"])
        for k in SUM:
            assert np.array_equal(getattr(want, k), getattr(r, k)), k
    for e in ranks + [ref]:
        e.close()


@pytest.mark.parametrize("mode,p", [("csr", 0.01), ("dense", 0.3)])
def test_rccl_one_rank_matches_single_engine(gossip, mode, p):
    n = 1000
    topo, t_cut, ev = _inputs(gossip, n, p, 41, 7.0)
    m = gossip.MODE_DENSE if mode == "dense" else gossip.MODE_CSR
    ref = _engine(gossip, n, t_cut, topo, ev, m, 0)
    ref.run()
    ref.sync()
    e = _engine(gossip, n, t_cut, topo, ev, m, 0, part=(0, 1))
    e.connect_rccl(gossip.rccl_unique_id())
    e.run()
    e.sync()
    a, b = ref.stats(), e.stats()
    for k in SUM + ("peers", "sockets"):
        assert np.array_equal(getattr(a, k), getattr(b, k)), k
    e.close()
    ref.close()


def test_abort_refuses_further_steps(gossip):
    # gossip_engine_abort (a failing rank tears its partition down): the communicator is freed, so
    # every later step of the engine -- and every collective its thread would still issue -- must
    # fail with E_STATE instead of touching it
    n = 1000
    topo, t_cut, ev = _inputs(gossip, n, 0.01, 41, 7.0)
    e = _engine(gossip, n, t_cut, topo, ev, gossip.MODE_CSR, 0, part=(0, 1))
    e.connect_rccl(gossip.rccl_unique_id())
    e.run(e.first_tick + 50)
    e.sync()
    e.abort()
    e.abort()  # idempotent
    with pytest.raises(gossip.GossipError, match="aborted") as ex:
        e.run()
    assert ex.value.code == gossip.E_STATE
    e.close()
    # without a communicator: host-staged stepping and the lockstep backend refuse it too
    topo2, t_cut2, ev2 = _inputs(gossip, 1100, 0.02, 51, 6.0)
    ranks = [_engine(gossip, 1100, t_cut2, topo2, ev2, gossip.MODE_CSR, 0, part=(r, 2)) for r in range(2)]
    ranks[1].abort()
    with pytest.raises(gossip.GossipError, match="aborted"):
        gossip.group_run(ranks)
    with pytest.raises(gossip.GossipError, match="aborted"):
        ranks[1].tick_begin()
    for r in ranks:
        r.close()


def test_row_partition_needs_an_exchange(gossip):
    n = 1100
    topo, t_cut, ev = _inputs(gossip, n, 0.02, 51, 6.0)
    e = _engine(gossip, n, t_cut, topo, ev, gossip.MODE_CSR, 0, part=(0, 2))
    with pytest.raises(gossip.GossipError, match="connect_rccl or gossip_engine_group_run"):
        e.run()
    e.close()
    e = gossip.Engine(400, L, T0, t_cut)  # blocks of 512 rows: rank 1 of 2 would own nothing
    e.set_row_partition(1, 2)
    with pytest.raises(gossip.GossipError, match="512-row block"):
        e.set_topology(gossip.Topology.gnp(400, 0.02, 1, gossip.TOPO_EXACT))
    e.close()


def test_xchunks_mismatch_is_refused(gossip):
    n = 1100
    topo, t_cut, ev = _inputs(gossip, n, 0.02, 51, 6.0)
    ranks = [_engine(gossip, n, t_cut, topo, ev, gossip.MODE_CSR, 0, part=(r, 2)) for r in range(2)]
    ranks[0].set_option("xchunks", 2)
    ranks[1].set_option("xchunks", 3)
    with pytest.raises(gossip.GossipError, match="different xchunks"):
        gossip.group_run(ranks)
    with pytest.raises(gossip.GossipError, match="xchunks"):
        ranks[0].set_option("xchunks", 17)
    for e in ranks:
        e.close()


@pytest.mark.parametrize("mode,p", [("csr", 0.01), ("dense", 0.3)])
def test_hybrid_share_shards_by_row_ranks(gossip, mode, p):
    # S share shards x R row ranks (the layout a 10M-node row rank needs to fit one
    # card): the ranks of each share shard run one row partition (lockstep backend); every rank
    # holds only its own rows of seen.  The S x R engines' counters sum to the single engine's,
    # with id collisions (groups stay inside one share shard).
    n, S, R = 2100, 2, 3  # (512-row blocks: ranks own 1024, 1024 and 52 rows)
    topo = gossip.Topology.gnp(n, p, 61, gossip.TOPO_EXACT)
    t_cut = gossip.seconds_to_ns(7.1)
    ev = gossip.make_schedule(n, 62, T0, t_cut, id_mask=0x7FFF if mode == "csr" else 0)
    m = gossip.MODE_DENSE if mode == "dense" else gossip.MODE_CSR
    ref = _engine(gossip, n, t_cut, topo, ev, m, 0)
    ref.run()
    ref.sync()
    want = ref.stats()
    ref.close()
    parts = []
    for s in range(S):
        ranks = []
        for r in range(R):
            e = gossip.Engine(n, L, T0, t_cut, mode=m, shard_rank=s, shard_count=S)
            e.set_row_partition(r, R)
            e.set_topology(topo)
            e.set_schedule(ev)
            ranks.append(e)
        gossip.group_run(ranks)
        for e in ranks:
            e.sync()
            parts.append(e.stats())
            c = e.counters()
            e.close()
    for k in SUM:
        total = sum(getattr(g, k).astype(np.uint64) for g in parts)
        assert np.array_equal(total, getattr(want, k).astype(np.uint64)), k


def test_rehearse_rows_keeps_results(gossip):
    # option rehearse_rows (one GPU stands in for one rank of an R-rank partition: per-block pull
    # launches, every block's rows packed and unpacked again) must not change a single counter
    n = 5000
    topo, t_cut, ev = _inputs(gossip, n, 0.004, 81, 6.6)
    want = _engine(gossip, n, t_cut, topo, ev, gossip.MODE_CSR, 0)
    want.run()
    w = want.stats()
    want.close()
    e = gossip.Engine(n, L, T0, t_cut, flags=gossip.F_TIMING)
    e.set_option("rehearse_rows", 3)
    e.set_topology(topo)
    e.set_schedule(ev)
    e.reset_timing()
    e.run()
    e.sync()
    got = e.stats()
    rh = e.rehearsal(3)
    e.close()
    for k in SUM + ("peers", "sockets"):
        assert np.array_equal(getattr(got, k), getattr(w, k)), k
    assert rh["ticks"] > 100 and (rh["pull_ms"] > 0).all() and (rh["msg_bytes"] > 0).all()
    assert (rh["pack_ms"] > 0).all() and (rh["unpack_ms"] > 0).all()
    # a rehearsal engine is unpartitioned: set_row_partition after the option is refused too
    e = gossip.Engine(n, L, T0, t_cut)
    e.set_option("rehearse_rows", 3)
    with pytest.raises(gossip.GossipError, match="rehearse_rows"):
        e.set_row_partition(0, 2)
    e.close()
