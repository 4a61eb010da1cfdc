"""World-size-2 rehearsal of the multi-GPU path on CPU (gloo).

Each rank takes the share instances `gossip_shard_events` gives it, simulates only those
(here with ORACLE A standing in for its GPU engine), and the ranks all-reduce the per-node
counters with the same helper bench.py uses.  The sum must equal a single full simulation
bit for bit -- including with forced id collisions, where instances must not be split.
"""
import os
import socket

import numpy as np
import pytest

from conftest import PKG, ROOT

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, q, id_mask):
    import sys

    sys.path.insert(0, PKG)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import torch.distributed as dist

    import gossip
    import gossip.dist as gd
    import oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        n, L, T0 = 400, 5_000_000, 5_000_000_000
        t_cut = gossip.seconds_to_ns(12.0)
        topo = gossip.Topology.gnp(n, 0.02, 5, gossip.TOPO_EXACT)
        ev = gossip.make_schedule(n, 99, T0, t_cut, id_mask=id_mask)
        owner = gossip.shard_events(topo, ev, WORLD)
        mine = ev[owner == rank]
        a, b = topo.links()
        r = oracle.run_replay(n, L, T0, t_cut, a, b, mine["ns"], mine["node"], mine["share_id"])
        st = gossip.Stats(r.gen, r.recv, r.fwd, r.sent, r.processed, r.peers, r.sockets)
        tot = gd.allreduce_stats(st)
        if rank == 0:
            full = oracle.run_replay(n, L, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"])
            ok = all(np.array_equal(getattr(tot, k), getattr(full, k))
                     for k in ("gen", "recv", "fwd", "sent", "processed", "peers", "sockets"))
            q.put((ok, int(len(mine)), int(len(ev))))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("id_mask", [0, 0x3FF])
def test_share_sharding_gloo_world2(id_mask):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, id_mask)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    ok, mine, total = q.get(timeout=5)
    assert 0 < mine < total
    assert ok
