#!/usr/bin/env python3
"""C5 on N GPUs with the row partition and the per-tick RCCL frontier exchange.

    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \\
        --master-port 29511 tools/bench_c5_rows.py [--width 4096] [--ticks 40]

One process per GPU; rank r owns a 512-row block of the 65,536 nodes, computes its rows of the
int8-MFMA contraction and exchanges its frontier rows with every other rank after each tick
(gossip_engine_connect_rccl: RCCL over xGMI).  The RCCL communicator id is made on rank 0 and
shared through torch.distributed (gloo).  Prints one JSON line on rank 0: whole-job edge
events/s over the timed flood (max wall over ranks), per-rank MFMA kernel time.  N = 1 runs the
same path on a 1-rank communicator."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "p2p-gossip-simulation-ns3_amd"))
import gossip  # noqa: E402

T0, L = 5_000_000_000, 5_000_000
INT8_PEAK_OPS = 5.0e15


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=4096)
    ap.add_argument("--ticks", type=int, default=40)
    ap.add_argument("--nodes", type=int, default=65536)
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")  # control plane only; the data path is RCCL in libgossip
    uid = gossip.rccl_unique_id() if rank == 0 else None
    if dist:
        box = [uid]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    n = a.nodes
    topo = gossip.Topology.gnp(n, 0.3, 5, gossip.TOPO_SKIP, threads=16)
    rng = np.random.Generator(np.random.Philox(12345))
    origins = rng.choice(n, size=a.width, replace=False)
    ev = gossip.events_from_arrays(np.full(a.width, T0 + 1000, np.int64), origins,
                                   np.arange(1, a.width + 1, dtype=np.uint32))
    t_cut = T0 + a.ticks * L
    eng = gossip.Engine(n, L, T0, t_cut, device=local, mode=gossip.MODE_DENSE, flags=gossip.F_TIMING)
    eng.set_row_partition(rank, world)
    eng.set_topology(topo)
    eng.set_schedule(ev)
    eng.connect_rccl(uid)
    eng.reset_timing()
    if dist:
        dist.barrier()
    eng.sync()
    t0 = time.perf_counter()
    eng.run()
    eng.sync()
    wall = time.perf_counter() - t0
    c = eng.counters()
    mine = np.array([c.edge_events, wall, c.pull_ms / max(c.pull_launches, 1),
                     c.dense_ops / (c.pull_ms * 1e-3) / INT8_PEAK_OPS if c.pull_ms else 0.0])
    if dist:
        import torch
        t = torch.tensor(mine, dtype=torch.float64)
        parts = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(parts, t)
        rows = np.stack([p.numpy() for p in parts])
    else:
        rows = mine[None, :]
    if rank == 0:
        edges = int(rows[:, 0].sum())
        tmax = float(rows[:, 1].max())
        print(json.dumps({
            "metric": "share-deliveries/sec (edge events)", "value": edges / tmax,
            "unit": "edge events/s", "n_gpus": world,
            "config": {"workload": f"C5: dense G(n,p) {n} nodes p=0.3, {a.width} concurrent shares, "
                                   f"row partition x{world}, RCCL frontier exchange per tick",
                       "ticks": c.ticks},
            "edge_events": edges, "wall_s_max": tmax,
            "per_rank_mfma_ms": rows[:, 2].tolist(), "per_rank_mfma_util": rows[:, 3].tolist()}),
            flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
