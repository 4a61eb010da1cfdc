#!/usr/bin/env python3
"""Benchmark: share-deliveries/sec (edge events/s) of the MI355X gossip engine.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = one tick (= --Latency = 5 ms of simulated time) of the tick-synchronous engine
over every live share column: the CSR pull over the bit-sliced frontier, dedup against the
seen bitmap, counters, and the new generations of that tick.

Workloads (BASELINE.json configs):
  N = 1  -> C3: sparse G(n,p), 1M nodes, average degree 16, 1 GPU (the largest single-GPU
            config; C4's full live window does not fit one GPU's HBM).
  N > 1  -> C4: sparse G(n,p), 10M nodes, average degree 16; share columns are sharded over
            the N ranks by share instance (no per-tick exchange, DESIGN.md "Multi-GPU"); the
            only collectives are the barrier and the final counter all-reduce over RCCL.
The timed window starts after W warm-up ticks from t = 5 s (the live window fills within
~10 ticks) and covers K ticks of steady-state gossip.  Inputs are resident in HBM before
the timed region starts.  `value` = edge events processed by all ranks / max-rank time.

The rank-0 N=1 run also times ORACLE A (the reference's P2PNode logic on one CPU core,
event-driven, unordered_set seen-sets) on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "p2p-gossip-simulation-ns3_amd"))

import numpy as np  # noqa: E402

import gossip  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
T0_NS = 5_000_000_000
SLICE_NS = 10_000_000_000  # steady-state slice start (tick 2000 at 5 ms)
L_NS = 5_000_000
T_CUT_NS = 59_900_000_000


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def workload(n_gpus):
    if n_gpus == 1:
        return dict(name="C3", nodes=1_000_000, desc="C3: sparse G(n,p), 1M nodes, avg degree 16, "
                    "5 ms ticks, 1 GPU", topo_seed=3, node_seed=1000)
    return dict(name="C4", nodes=10_000_000, desc="C4: sparse G(n,p), 10M nodes, avg degree 16, "
                "5 ms ticks, share-sharded over GPUs", topo_seed=4, node_seed=2000)


def pmc_traffic(name, n_gpus):
    """HBM bytes per pull launch from a committed rocprofv3 PMC pass of this bench command
    (profiles/pmc_<workload>.json, written by tools/pmc_traffic.py), or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{name}.json")
    if n_gpus != 1 or not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            return float(json.load(f)["hbm_bytes_per_launch"])
    except Exception:
        return None


def cpu_baseline(topo, ev, sample_shares, threads):
    """ORACLE A (single thread) on the first `sample_shares` generations of the workload,
    floods run to completion.  Test infrastructure used only as the timed CPU baseline."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    a, b = topo.links()
    sub = ev[:sample_shares]
    r = oracle.run_replay(topo.num_nodes, L_NS, SLICE_NS, oracle.INT64_MAX, a, b, sub["ns"],
                          sub["node"], sub["share_id"])
    return dict(value=r.edge_events / r.wall_s if r.wall_s > 0 else None, unit="edge events/s",
                cores=1, kind="port",
                sample=f"ORACLE A (event-driven P2PNode logic, unordered_set seen-sets) on the "
                       f"same graph, the first {len(sub)} generations after t=10 s, floods run "
                       f"to completion: {r.edge_events} edge events in {r.wall_s:.2f} s "
                       f"(host nproc {os.cpu_count()}, threads=1)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=2)
    ap.add_argument("--noskip", action="store_true",
                    help="diagnostic: dense pull (every peer-row word read) for PMC calibration")
    ap.add_argument("--pull-kernel", choices=("auto", "wide", "generic"), default="auto",
                    help="diagnostic: force the scalar-peer (wide) or lane-shuffle (generic) pull")
    ap.add_argument("--rehearse-shards", type=int, default=0,
                    help="diagnostic: run only shard 0 of S on this one GPU (per-rank footprint "
                         "and time of an S-GPU run); the JSON line is marked REHEARSAL")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = args.gpus
    dist = None
    dev = None
    if world > 1:
        import torch
        import torch.distributed as dist

        # GOSSIP_DIST_BACKEND=gloo + GOSSIP_BENCH_NODES: rehearsal of N ranks on one GPU.
        backend = os.environ.get("GOSSIP_DIST_BACKEND", "nccl")  # "nccl" = RCCL over xGMI
        local = local % max(torch.cuda.device_count(), 1)
        if backend == "nccl":
            torch.cuda.set_device(local)
            dev = f"cuda:{local}"
        dist.init_process_group(backend)
        import gossip.dist as gd
    wl = workload(n_gpus)
    if os.environ.get("GOSSIP_BENCH_NODES"):
        wl["nodes"] = int(os.environ["GOSSIP_BENCH_NODES"])
        wl["desc"] += f" [REHEARSAL: {wl['nodes']} nodes]"
    n = wl["nodes"]
    p = 16.0 / (n - 1)
    W, K = args.warmup, args.steps

    t_setup = time.time()
    topo = gossip.Topology.gnp(n, p, wl["topo_seed"], gossip.TOPO_SKIP, threads=args.threads)
    # Steady-state slice: the share schedule is the reference's (node RNGs from t = 0, ids
    # counted from t = 5 s); the slice starts at t = 10 s (tick 2000), where the U(2,5) s
    # renewal density has settled at 1/3.5 s per node (at t = 5 s it is only 1/9 s).
    t_gen_end = SLICE_NS + (W + K + 1) * L_NS
    ev = gossip.make_schedule(n, wl["node_seed"], T0_NS, T_CUT_NS, t_gen_end_ns=t_gen_end,
                              threads=args.threads)
    ev = ev[ev["ns"] >= SLICE_NS]
    shards = max(world, 1)
    if args.rehearse_shards > 1 and world == 1:
        shards = args.rehearse_shards
        wl["desc"] += f" [REHEARSAL: shard 0 of {shards} on one GPU]"
    flags = gossip.F_TIMING | (gossip.F_NOSKIP if args.noskip else 0)
    flags |= {"auto": 0, "wide": gossip.F_WIDE_PULL, "generic": gossip.F_GENERIC_PULL}[args.pull_kernel]
    eng = gossip.Engine(n, L_NS, SLICE_NS, T_CUT_NS, device=local, flags=flags,
                        shard_rank=rank, shard_count=shards)
    eng.set_topology(topo)
    eng.set_schedule(ev)
    if rank == 0:
        rp, _, _ = topo.csr()
        log(f"[bench] {wl['desc']}: {topo.num_nodes} nodes, {int(rp[-1])} directed entries, "
            f"{len(ev)} generations in window, setup {time.time() - t_setup:.1f} s")

    tick0 = eng.first_tick
    eng.run(tick0 + W)
    eng.sync()
    c0 = eng.counters()
    eng.reset_timing()
    if dist:
        dist.barrier()
    eng.sync()
    t0 = time.perf_counter()
    eng.run(tick0 + W + K)
    eng.sync()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    c1 = eng.counters()
    edges = c1.edge_events - c0.edge_events
    pull_ms, pull_bytes, launches = c1.pull_ms, c1.pull_bytes, c1.pull_launches
    gens_done = c1.generations
    if dist:
        elapsed, pull_ms_max = gd.allreduce_scalars([elapsed, pull_ms], op="max", device=dev)
        edges_total, gens_total = gd.allreduce_scalars([edges, gens_done], op="sum", device=dev)
        edges_total = int(edges_total)
        # every counted generation of the simulated ticks ran on exactly one rank
        want = int(np.count_nonzero(ev["ns"] < (tick0 + W + K) * L_NS))
        if int(gens_total) != want:
            raise SystemExit(f"shard coverage broken: {int(gens_total)} generations vs {want}")
    else:
        edges_total = edges
        pull_ms_max = pull_ms

    if rank == 0:
        avg_ms = pull_ms / max(launches, 1)
        # Algorithmic bytes per launch of the implemented pull: 16 B per
        # (edge, word-pair) neighbour read actually needed + 4 B per col index of a pulling
        # node pass + 16 B per own-row seen/F access + 24 B of per-node row_ptr/counters.
        bytes_per_launch = c1.pull_bytes_moved / max(launches, 1)
        dense_bytes_per_launch = pull_bytes / max(launches, 1)  # SURVEY §8d dense formula
        achieved = bytes_per_launch / (avg_ms * 1e6) if avg_ms > 0 else 0.0  # GB/s
        traffic = pmc_traffic(wl["name"], n_gpus)
        per_launch = lambda x: float(x) / max(launches, 1)  # noqa: E731
        out = {
            "metric": "share-deliveries/sec (edge events)",
            "value": edges_total / elapsed,
            "unit": "edge events/s",
            "n_gpus": n_gpus,
            "steps": K,
            "warmup": W,
            "ms_per_step": elapsed * 1e3 / K,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic: G(n,p) by Philox geometric skipping + the reference's mt19937 "
                    "share schedule (node seed + id)",
            "config": {
                "workload": wl["desc"],
                "nodes": n,
                "avg_degree": 16,
                "latency_ms": 5,
                "ticks_timed": [tick0 + W, tick0 + W + K],
                "edge_events_timed": edges_total,
                "live_words_per_node": c1.words_hw,
                "window_capacity_words": c1.words_cap,
                "device_gib": c1.device_bytes / 2**30,
                "parallelism": f"share-shard x{shards}",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "k_pull",
                "bytes_per_launch": bytes_per_launch,
                "dense_formula_bytes_per_launch": dense_bytes_per_launch,
                "dense_formula_equiv_gbs": (dense_bytes_per_launch / (avg_ms * 1e6)) if avg_ms > 0 else None,
                "avg_launch_ms": avg_ms,
                "bytes_breakdown_per_launch": {
                    "peer_rows": per_launch(16 * c1.pull_pair_edges),
                    "peer_ids": per_launch(4 * c1.pull_col_ids),
                    "peer_occupancy": per_launch(8 * c1.pull_nz_reads),
                    "own_seen_read": per_launch(16 * c1.pull_seen_reads),
                    "own_seen_write": per_launch(16 * c1.pull_seen_writes),
                    "frontier_write": per_launch(16 * c1.pull_f_writes),
                    "per_node_rowptr_counters_occupancy": per_launch(
                        c1.pull_bytes_moved - 16 * c1.pull_pair_edges - 4 * c1.pull_col_ids -
                        8 * c1.pull_nz_reads - 16 * (c1.pull_seen_reads + c1.pull_seen_writes +
                                                     c1.pull_f_writes)),
                },
                "pull_fraction_of_step": (pull_ms_max / (elapsed * 1e3)) if elapsed > 0 else None,
            },
        }
        if n_gpus == 1 and world == 1 and not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(topo, ev, args.cpu_sample, args.threads)
            except Exception as e:  # the baseline is reported, never required
                out["cpu_baseline"] = {"value": None, "error": str(e)}
        print(json.dumps(out), flush=True)
    eng.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
