"""World-size-2 runs of the PRODUCT's multi-GPU paths, one process per rank (both on the one GPU
of the test box; torch.distributed gloo as the transport / control plane):

* share shards: each process runs libgossip's engine for shard r of 2 and the ranks all-reduce
  the per-node counters (gossip.dist, the helper bench.py uses);
* row partition with the host-staged exchange: each process owns a block of node rows and, every
  tick, exports its packed occupied frontier rows (gossip_engine_exchange_export), all-gathers
  the messages over gloo and imports the other rank's (the same messages the RCCL backend
  broadcasts over xGMI);
* the same, pipelined ("rows-*-chunked"): per row chunk, export_chunk waits only for that chunk
  of the GPU's pull, so chunk c travels while the GPU pulls chunk c + 1 -- the RCCL backend's
  overlap, on the engine's exchange stream.

Both must sum to the single engine's counters bit for bit, with forced id collisions for the
shards and the dense (MFMA) path for the rows.
"""
import os
import socket

import numpy as np
import pytest

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

WORLD = 2
SUM = ("gen", "recv", "fwd", "sent", "processed")
L, T0 = 5_000_000, 5_000_000_000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(gossip, case):
    if case == "shards":
        n = 3000
        topo = gossip.Topology.gnp(n, 10.0 / (n - 1), 21, gossip.TOPO_SKIP)
        t_cut = gossip.seconds_to_ns(9.0)
        ev = gossip.make_schedule(n, 22, T0, t_cut, id_mask=0x3FFF)
        return n, topo, t_cut, ev, gossip.MODE_CSR
    n = 2048 if not case.endswith("chunked") else 4096
    dense = case.startswith("rows-dense")
    topo = gossip.Topology.gnp(n, 0.3 if dense else 0.01, 23, gossip.TOPO_EXACT)
    t_cut = gossip.seconds_to_ns(6.3)
    ev = gossip.make_schedule(n, 24, T0, t_cut)
    return n, topo, t_cut, ev, (gossip.MODE_DENSE if dense else gossip.MODE_CSR)


def _worker(rank, port, q, case):
    import sys

    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist

    import gossip
    import gossip.dist as gd

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        n, topo, t_cut, ev, mode = _inputs(gossip, case)
        if case == "shards":
            eng = gossip.Engine(n, L, T0, t_cut, mode=mode, shard_rank=rank, shard_count=WORLD)
            eng.set_topology(topo)
            eng.set_schedule(ev)
            eng.run()
            eng.sync()
            out = gd.allreduce_stats(eng.stats())
            sent = recvd = 0
        else:
            eng = gossip.Engine(n, L, T0, t_cut, mode=mode)
            eng.set_row_partition(rank, WORLD)
            eng.set_topology(topo)
            eng.set_schedule(ev)
            chunked = case.endswith("chunked")
            if chunked:
                eng.set_option("xchunks", 3)
                assert eng.exchange_chunks() == 3
            ticks = 0
            while eng.tick_begin():
                for c in range(eng.exchange_chunks() if chunked else 1):
                    mine = eng.exchange_export_chunk(c) if chunked else eng.exchange_export()
                    msgs = [None] * WORLD
                    dist.all_gather_object(msgs, mine)
                    for r in range(WORLD):
                        if r != rank:
                            if chunked:
                                eng.exchange_import_chunk(r, c, msgs[r])
                            else:
                                eng.exchange_import(r, msgs[r])
                eng.tick_end()
                ticks += 1
            eng.sync()
            out = gd.allreduce_stats(eng.stats())
            c = eng.counters()
            sent, recvd = c.exchange_bytes_sent, c.exchange_bytes_received
        eng.close()
        if rank == 0:
            q.put(({k: getattr(out, k) for k in SUM}, sent, recvd))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", ["shards", "rows-csr", "rows-dense", "rows-csr-chunked", "rows-dense-chunked"])
def test_world2_processes_match_single_engine(gossip, case):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, case)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got, sent, recvd = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n, topo, t_cut, ev, mode = _inputs(gossip, case)
    eng = gossip.Engine(n, L, T0, t_cut, mode=mode)
    eng.set_topology(topo)
    eng.set_schedule(ev)
    eng.run()
    want = eng.stats()
    c = eng.counters()
    eng.close()
    for k in SUM:
        assert np.array_equal(got[k].astype(np.uint64), getattr(want, k).astype(np.uint64)), k
    if case != "shards":
        # the exchange moved only occupied tile rows: far less than whole F_next row blocks
        full = c.ticks * (n // 2) * c.words_cap * 8
        assert 0 < sent < full and 0 < recvd < full
