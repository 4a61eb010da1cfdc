"""Multi-GPU plumbing: one process per GPU, share-instance shards, counters summed at the end.

The engine needs no per-tick exchange: each rank simulates the share
instances `gossip_shard_events` assigns to it, on its own device, over the whole graph.  The
only collectives are a barrier around the timed region and the final reduction of the
per-node counters -- torch.distributed over RCCL ("nccl") on GPUs, "gloo" in the CPU tests.
"""
from __future__ import annotations

import numpy as np

from . import Stats

ADDITIVE = ("gen", "recv", "fwd", "sent", "processed")


def allreduce_stats(st: Stats, device=None) -> Stats:
    """Sum the additive per-node counters over all ranks (peers/sockets are per-graph and
    identical on every rank, so they are kept as they are)."""
    import torch
    import torch.distributed as dist

    out = {}
    for k in ADDITIVE:
        a = getattr(st, k)
        t = torch.from_numpy(a.astype(np.int64))
        if device is not None:
            t = t.to(device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        v = t.cpu().numpy()
        out[k] = v.astype(np.uint64) if k == "sent" else v.astype(np.uint32)
    return Stats(out["gen"], out["recv"], out["fwd"], out["sent"], out["processed"],
                 st.peers.copy(), st.sockets.copy())


def allreduce_scalars(values, op="sum", device=None):
    import torch
    import torch.distributed as dist

    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu().tolist()]
