#!/usr/bin/env python3
"""Benchmark: share-deliveries/sec (edge events/s) of the MI355X gossip engine.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload C4|C3]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

One step = one tick (= --Latency = 5 ms of simulated time) of the tick-synchronous engine
over every live share column: the CSR pull over the bit-sliced frontier, dedup against the
seen bitmap, counters, and the new generations of that tick.

Workload (BASELINE.json metric: "share-deliveries/sec at 10M nodes, 1/2/4/8 GPUs"):
  C4: sparse G(n,p), 10M nodes, average degree 16, every share generated in the window.
The share columns are split into share-instance shards (gossip_shard_events; no per-tick
exchange, DESIGN.md "Multi-GPU").  C4's live window needs two shards' worth of HBM (one shard
holds ~265 GiB of bitmaps), so the job is always cut into max(2, N) shards: at N = 1 the one
GPU runs shard 0 and then shard 1 (each with its own warm-up, timed separately, the times
added); at N >= 2 every rank runs one shard.  The total work is the same at every N
(strong scaling); the only collectives are barriers and the final scalar reductions (RCCL).
--workload C3 (1M nodes, one shard per GPU) is kept for kernel A/B work.

The timed window of a shard starts after W warm-up ticks from t = 10 s and covers K ticks of
steady-state gossip; inputs are resident in HBM before it starts.
`value` = edge events processed by all shards / (max over ranks of the rank's summed timed
windows).

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
import gossip.workloads as WL  # noqa: E402

# BASELINE.json "metric", quoted on C4 (10M nodes)
BASELINE_METRIC = "share-deliveries/sec (edge events) at 10M nodes, 1/2/4/8 GPUs; % HBM/MFMA peak"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
# Every engine option that shapes the pull launches (include/gossip.h), read back from the engine
# and recorded in the line's pull_variant: committed PMC traffic attaches only to a line whose
# variant -- these values, the resolved young grid and the library build -- equals the pass's
LAUNCH_OPTIONS = ("pull_nt", "pull_grid", "pull_gate", "pull_tiles", "pull_tile_order",
                  "pull_sat", "dense_rows", "late_age", "young", "young_age", "young_cap",
                  "young_list_cap", "young_nt", "young_overlap", "young_grid", "young_skip")


def option_or_none(eng, name):
    """An engine option's value, or None when the loaded library predates the option (A/B runs
    against an earlier build)."""
    try:
        return eng.get_option(name)
    except gossip.GossipError:
        return None


def lib_build_id():
    """sha256 (first 16 hex digits) of the libgossip.so this process loaded."""
    import hashlib
    with open(gossip.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]
T0_NS = 5_000_000_000
SLICE_NS = 10_000_000_000  # steady-state slice start (tick 2000 at 5 ms)
L_NS = 5_000_000
T_CUT_NS = 59_900_000_000

WORKLOADS = {
    # fit_shards: share shards one GPU's HBM must be cut into for the live window to fit (the
    # bench doubles it on its own when an engine reports GOSSIP_ECAPACITY / GOSSIP_ENOMEM)
    "C4": dict(fit_shards=2, desc="C4: sparse G(n,p), 10M nodes, avg degree 16, 5 ms ticks"),
    "C3": dict(fit_shards=1, desc="C3: sparse G(n,p), 1M nodes, avg degree 16, 5 ms ticks"),
}
CAPACITY_CODES = (-3, -5)  # GOSSIP_ENOMEM, GOSSIP_ECAPACITY


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pmc_traffic(name, line, variant):
    """HBM bytes per pull launch from the committed rocprofv3 PMC pass of this workload
    (profiles/pmc_<workload>.json, written by tools/pmc_traffic.py), only when that pass ran the
    same configuration as this line; otherwise (None, reason)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{name}.json")
    if line["n_gpus"] != 1:
        return None, "PMC pass is single-GPU"
    if not os.path.exists(path):
        return None, f"no {os.path.relpath(path, ROOT)}"
    try:
        with open(path) as f:
            d = json.load(f)
    except Exception as e:  # a malformed file is reported, not fatal
        return None, f"unreadable PMC file: {e}"
    cfg = d.get("config") or {}
    want = {"workload": name.split("_")[0], "warmup": line["warmup"], "steps": line["steps"],
            "live_words_per_node": line["config"]["live_words_per_node"],
            "pull_variant": variant}
    diff = {k: (cfg.get(k), v) for k, v in want.items() if cfg.get(k) != v}
    if diff:
        return None, f"PMC pass config differs from this line: {diff}"
    return float(d["hbm_bytes_per_launch"]), None


def cpu_baseline(topo, ev, sample_shares, hops):
    """ORACLE A (single thread) on the first `sample_shares` generations of the workload's
    steady-state slice, their floods cut after `hops` hops (PrintStatistics time).  Test
    infrastructure used only as the timed CPU baseline."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    a, b = topo.links()
    sub = ev[:sample_shares]
    t_cut = int(sub["ns"].max()) + hops * L_NS + 1 if hops > 0 else oracle.INT64_MAX
    r = oracle.run_replay(topo.num_nodes, L_NS, SLICE_NS, t_cut, a, b, sub["ns"], sub["node"],
                          sub["share_id"])
    cut = f"cut after {hops} hops" if hops > 0 else "run to completion"
    return dict(value=r.edge_events / r.wall_s if r.wall_s > 0 else None, unit="edge events/s",
                cores=1, kind="port",
                sample=f"ORACLE A (event-driven P2PNode logic, hash-set seen-sets) on the "
                       f"same graph, the first {len(sub)} generation(s) after t=10 s, floods "
                       f"{cut}: {r.edge_events} edge events in {r.wall_s:.2f} s of event loop "
                       f"(host nproc {os.cpu_count()}, threads=1)")


def cpu_baseline_bitsliced(topo, ev, sample_shares, hops, threads):
    """ORACLE B (bit-sliced, level-synchronous, multithreaded CPU restatement; SURVEY 8(d)'s
    optional all-cores baseline, reported beside the single-core ORACLE A one): the first
    `sample_shares` generations of the slice (distinct ids), floods cut after `hops` hops; the
    timer covers the propagation, not the CSR construction."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    a, b = topo.links()
    sub = ev[:sample_shares]
    sub = sub[np.unique(sub["share_id"], return_index=True)[1]]  # distinct ids (ORACLE B's domain)
    sub = sub[np.lexsort((sub["node"], sub["ns"]))]
    t_cut = int(sub["ns"].max()) + hops * L_NS + 1
    r = oracle.run_oracle_b(topo.num_nodes, L_NS, t_cut, a, b, sub["ns"], sub["node"], sub["share_id"],
                            threads=threads)
    return dict(value=r.edge_events / r.wall_s if r.wall_s > 0 else None, unit="edge events/s",
                cores=threads, kind="port",
                sample=f"ORACLE B (bit-sliced 64 shares per word, level-synchronous, {threads} threads) "
                       f"on the same graph, the first {len(sub)} generations after t=10 s, floods "
                       f"cut after {hops} hops: {r.edge_events} edge events in {r.wall_s:.2f} s of "
                       f"propagation (host nproc {os.cpu_count()})")


def young_breakdown(acc, launches, n):
    """k_pull_young's algorithmic bytes per launch, item by item: the terms of the engine's
    young_bytes_moved (engine.hip, gossip_engine_get_counters), so the items add up to
    bytes_per_launch (tests/test_bench_pmc.py)."""
    yl = max(launches, 1)
    return {
        "slot_lines_read": 128 * acc["young_sl"] / yl,
        "fallback_rows_read": 128 * acc["young_fb"] / yl,
        "peer_ids_and_hints": 5 * acc["young_col_ids"] / yl,
        "own_seen_read": 8 * acc["young_seen_reads"] / yl,
        "own_seen_write": 8 * acc["young_seen_writes"] / yl,
        "dense_rows_written": 128 * acc["young_rows_written"] / yl,
        "slot_lines_written": 128 * acc["young_slot_writes"] / yl,
        "unhinted_second_lines_read": 128 * acc.get("young_line2_misses", 0) / yl,
        # seen rows written whole: the lists of tiles leaving the young set materialised, and
        # fresh tiles cleared at nodes whose list overflowed (young_fresh_lines)
        "seen_rows_written_whole": 128 * acc.get("young_fresh_lines", 0) / yl,
        "seen_list_lines_read_written": 128 * acc.get("young_list_lines", 0) / yl,
        "per_node_rowptr_counters": 8.0 * (n + 1) + 16.0 * n,
    }


def run_shards(args, wl, topo, ev, my_shards, shards, dist, dev, local, rank, flags):
    """Warm up and time every shard this rank owns; raises gossip.GossipError on failure."""
    W, K = args.warmup, args.steps
    slice_tick = SLICE_NS // L_NS
    acc = dict(elapsed=0.0, edges=0, gens=0, launches=0, pull_ms=0.0, moved=0, dense=0, pe=0,
               col=0, nz=0, srd=0, swr=0, fwr=0, words_hw=0, words_cap=0, dev_bytes=0, nt=0,
               grid=0, ramp_ticks=0, young_ms=0.0, young_launches=0, young_bytes=0, young_sl=0,
               young_fb=0, phase_ms=0.0)
    for s in my_shards:
        t_eng = time.perf_counter()
        eng = gossip.Engine(wl["nodes"], L_NS, T0_NS, T_CUT_NS, device=local, flags=flags,
                            shard_rank=s, shard_count=shards)
        acc["options"] = {k: option_or_none(eng, k) for k in LAUNCH_OPTIONS}
        try:
            eng.set_topology(topo)
            eng.set_schedule(ev)
            # ramp: every tick from the first generation of the slice schedule (LIFE ticks before
            # t = 10 s, plus the earlier floods of ids that recur in it) through W warm-up ticks
            eng.run(slice_tick + W)
            eng.sync()
            c0 = eng.counters()
            eng.reset_timing()
            if dist:
                dist.barrier()
            eng.sync()
            t0 = time.perf_counter()
            eng.run(slice_tick + W + K)
            eng.sync()
            if dist:
                dist.barrier()
            t1 = time.perf_counter()
            c1 = eng.counters()
        finally:
            eng.close()
        acc["elapsed"] += t1 - t0
        acc["edges"] += c1.edge_events - c0.edge_events
        acc["gens"] += c1.generations
        acc["pull_ms"] += c1.pull_ms
        acc["launches"] += c1.pull_launches
        for k, f in (("moved", "pull_bytes_moved"), ("dense", "pull_bytes"), ("pe", "pull_pair_edges"),
                     ("col", "pull_col_ids"), ("nz", "pull_nz_reads"), ("srd", "pull_seen_reads"),
                     ("swr", "pull_seen_writes"), ("fwr", "pull_f_writes")):
            acc[k] += getattr(c1, f)
        acc["young_ms"] += c1.young_ms
        acc["young_launches"] += c1.young_launches
        acc["young_bytes"] += c1.young_bytes_moved
        acc["young_sl"] += c1.young_slot_lines
        acc["young_fb"] += c1.young_fallback_rows
        for k in ("young_col_ids", "young_seen_reads", "young_seen_writes", "young_rows_written",
                  "young_slot_writes", "young_line2_misses", "young_fresh_lines", "young_list_lines"):
            acc[k] = acc.get(k, 0) + getattr(c1, k)
        acc["phase_ms"] += c1.pull_phase_ms
        acc["words_hw"] = max(acc["words_hw"], c1.words_hw)
        acc["words_cap"] = max(acc["words_cap"], c1.words_cap)
        acc["dev_bytes"] = max(acc["dev_bytes"], c1.device_bytes)
        acc["nt"], acc["grid"] = c1.pull_nt, c1.pull_grid
        acc["late_age"] = c1.pull_late_age
        acc["pull_tiles"] = c1.pull_tiles
        acc["lpw"], acc["pull_sat"] = c1.pull_lpw, c1.pull_sat
        acc["young_grid"] = c1.young_grid
        acc["dense_tiles"] = max(acc.get("dense_tiles", 0), c1.pull_dense_tiles)
        # (device-side tallies restart at reset_timing: c1 holds the timed ticks alone)
        acc["sat_skips"] = acc.get("sat_skips", 0) + c1.pull_sat_skips
        acc["items"] = acc.get("items", 0) + c1.pull_items
        acc["gather_items"] = acc.get("gather_items", 0) + c1.pull_gather_items
        acc["early_retires"] = acc.get("early_retires", 0) + c1.window_early_retires
        acc["ramp_ticks"] = c0.ticks
        if rank == 0:
            log(f"[bench] shard {s} of {shards}: {c1.edge_events - c0.edge_events} edge events in "
                f"{(t1 - t0) * 1e3:.1f} ms, window {c1.words_hw} words, ramp {c0.ticks} ticks, "
                f"engine setup + ramp {t0 - t_eng:.1f} s")
    return acc


def rehearse_rows(args, wl, topo, ev, shards, R, flags):
    """One GPU, share shard 0 of `shards`, run as the R row blocks of a row partition would run it
    (engine option rehearse_rows; young tiles off, as on a row rank): per block and timed tick,
    the pull over the block's rows, the pack of its F_next rows into its exchange message, the
    unpack of that message (the work each OTHER rank does for it) and the message bytes.  A rank's
    tick then costs its own pull + pack + the unpacks of the R - 1 other blocks, and it receives
    the R - 1 other messages over xGMI.  Prints one JSON line marked REHEARSAL."""
    W, K = args.warmup, args.steps
    slice_tick = SLICE_NS // L_NS
    eng = gossip.Engine(wl["nodes"], L_NS, T0_NS, T_CUT_NS, flags=flags, shard_rank=0, shard_count=shards)
    try:
        eng.set_option("young", 0)
        eng.set_option("rehearse_rows", R)
        eng.set_topology(topo)
        eng.set_schedule(ev)
        eng.run(slice_tick + W)
        eng.sync()
        eng.reset_timing()
        c0 = eng.counters()
        t0 = time.perf_counter()
        eng.run(slice_tick + W + K)
        eng.sync()
        wall = time.perf_counter() - t0
        c1 = eng.counters()
        rh = eng.rehearsal(R)
    finally:
        eng.close()
    T = max(rh["ticks"], 1)
    pull, pack, unpack = rh["pull_ms"] / T, rh["pack_ms"] / T, rh["unpack_ms"] / T
    msg = rh["msg_bytes"].astype(np.float64) / T
    rank_ms = pull + pack + (unpack.sum() - unpack)  # own pull + own pack + the others' unpacks
    ingress = msg.sum() - msg
    n = wl["nodes"]
    own_rows = np.diff(np.minimum(np.arange(R + 1) * (((n + R - 1) // R + 511) // 512 * 512), n))
    fbytes = 2 * n * c1.words_cap * 8
    out = {
        "metric": "REHEARSAL: row partition, one rank's work per tick (not a throughput)",
        "workload": f"{wl['desc']}, share shard 0 of {shards}, row blocks of an R = {R} partition, "
                    f"{K} timed ticks after {W} warm-up from t = 10 s, young tiles off",
        "rows_per_rank": own_rows.tolist(),
        "edge_events_per_tick_whole_shard": (c1.edge_events - c0.edge_events) / T,
        "pull_ms_per_tick": pull.tolist(),
        "pack_ms_per_tick": pack.tolist(),
        "unpack_ms_per_tick": unpack.tolist(),
        "message_bytes_per_tick": msg.tolist(),
        "rank_gpu_ms_per_tick": rank_ms.tolist(),
        "rank_gpu_ms_per_tick_max": float(rank_ms.max()),
        "rank_ingress_bytes_per_tick": ingress.tolist(),
        "rank_ingress_bytes_per_tick_max": float(ingress.max()),
        "unpartitioned_pull_ms_per_tick": c1.pull_ms / max(c1.pull_launches, 1),
        # + the exchange buffers a rank would hold: its own message and the R - 1 it receives, each
        # sized for the largest message of a tick (not the mean: ADVICE r04)
        "message_bytes_per_tick_max": rh["msg_bytes_max"].astype(np.float64).tolist(),
        "rank_device_gib": (fbytes + c1.words_cap * 8 * int(own_rows.max()) + R * float(rh["msg_bytes_max"].max())) / 2**30,
        "wall_s_rehearsal": wall,
        "window_words": c1.words_hw,
    }
    print(json.dumps(out), flush=True)


def resolve_shard_rule(rule, shards):
    """--shard-rule auto: the birth-tick rule from 8 share shards on, the hash rule below (one-rank
    rehearsals, DESIGN.md section 5: 8 shards 24.8 vs 27.6 ms per tick, 22.1 with the tick rule's
    fresh tile per birth tick (shard_flags); 4 shards 39.8 vs 36.7;
    2 shards: the tick rule's window peaks overflow the capacity estimate)."""
    return rule if rule != "auto" else ("tick" if shards >= 8 else "hash")


def shard_flags(rule, fresh="auto"):
    """Engine flags of a resolved shard rule.  The birth-tick rule also opens a fresh tile per
    birth tick (GOSSIP_F_TILE_PER_TICK): a shard's births of one tick then never share a tile with
    its births 8 ticks later, so every tile stays single-age -- young while its shares are young,
    one age for the early exit, saturation bits and dense rows (one rank of 8: 22.1 vs 24.8 ms per
    tick, same edge events).  The hash rule keeps the packed tiles (C4's 2
    shards: 58.67 vs 58.15 ms per shard-tick with fresh tiles)."""
    f = gossip.F_SHARD_BY_TICK if rule == "tick" else 0
    if fresh == "on" or (fresh == "auto" and rule == "tick"):  # (--fresh-tiles: A/B override)
        f |= gossip.F_TILE_PER_TICK
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="C4")
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1, help="generations in the CPU sample")
    ap.add_argument("--cpu-hops", type=int, default=6, help="hops the CPU-sample floods run")
    ap.add_argument("--noskip", action="store_true",
                    help="diagnostic: dense pull (every peer-row word read) for PMC calibration")
    ap.add_argument("--rehearse-shards", type=int, default=0,
                    help="diagnostic: run only shard 0 of S on this one GPU (per-rank footprint "
                         "and time of an S-GPU run); the JSON line is marked REHEARSAL")
    ap.add_argument("--shard-rule", choices=["auto", "hash", "tick"], default="auto",
                    help="share-shard rule: hash of the instance key, or the birth tick of its first "
                         "generation (GOSSIP_F_SHARD_BY_TICK: a shard's births of a tick fill whole "
                         "tiles of one age); auto (default): tick from 8 shards on, hash below "
                         "(DESIGN.md section 5: measured one-rank rehearsals)")
    ap.add_argument("--fresh-tiles", choices=["auto", "on", "off"], default="auto",
                    help="a fresh tile per birth tick (GOSSIP_F_TILE_PER_TICK); auto (default): with "
                         "the tick rule only (shard_flags)")
    ap.add_argument("--rehearse-index", type=int, default=0,
                    help="diagnostic, with --rehearse-shards S: the shard (rank) to rehearse, or -1 for "
                         "every rank 0..S-1 one after another (the line then reports each rank's time "
                         "and the job's tick = the slowest rank's)")
    ap.add_argument("--rehearse-rows", type=int, default=0,
                    help="diagnostic: one rank of an R-rank row partition of share shard 0 of "
                         "--rehearse-shards (default: the workload's fit) on this one GPU")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rehearsal = (args.rehearse_shards > 1 or args.rehearse_rows > 1) and world == 1
    if args.gpus != world and not rehearsal:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N > 1 with "
                         f"torch.distributed.run (one process per GPU), or use --rehearse-shards")
    n_gpus = world
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
    wl = dict(WORKLOADS[args.workload], name=args.workload)
    wl["nodes"] = WL.CONFIGS[args.workload]["nodes"]
    if os.environ.get("GOSSIP_BENCH_NODES"):
        wl["nodes"] = int(os.environ["GOSSIP_BENCH_NODES"])
        wl["desc"] += f" [REHEARSAL: {wl['nodes']} nodes]"
    n = wl["nodes"]
    W, K = args.warmup, args.steps

    t_setup = time.time()
    topo = WL.topology(args.workload, nodes=n, threads=args.threads)
    # Steady-state slice of the reference's continuous run: the schedule is the reference's
    # (node RNGs from t = 0, ids counted from t = 5 s); the timed ticks start W ticks after
    # t = 10 s (tick 2000).  The engine replays every generation of the LIFE ticks before 10 s
    # and all earlier generations of the ids that occur in the slice (workloads.slice_schedule).
    t_gen_end = SLICE_NS + (W + K + 1) * L_NS
    ev, sinfo = WL.slice_schedule(n, WL.CONFIGS[args.workload]["node_seed"], SLICE_NS, t_gen_end,
                                  threads=args.threads)
    flags = gossip.F_TIMING | (gossip.F_NOSKIP if args.noskip else 0)

    def shard_rule(shards):
        return resolve_shard_rule(args.shard_rule, shards)
    if rank == 0:
        rp, _, _ = topo.csr()
        log(f"[bench] {wl['desc']}: {topo.num_nodes} nodes, {int(rp[-1])} directed entries, "
            f"{len(ev)} generations in the slice schedule ({sinfo['earlier_same_id']} earlier "
            f"generations of recurring ids), setup {time.time() - t_setup:.1f} s")

    if args.rehearse_rows > 1:
        rehearse_rows(args, wl, topo, ev, max(args.rehearse_shards, wl["fit_shards"]), args.rehearse_rows,
                      flags | gossip.F_TIMING)
        return
    # Shards: at least what one GPU's HBM needs, at least one per rank, a multiple of the ranks;
    # doubled (on every rank) when any rank's engine runs out of device memory.
    passes = max(1, -(-wl["fit_shards"] // world))
    retried = []  # share-shard counts that did not fit (GOSSIP_ECAPACITY / ENOMEM), in order
    while True:
        shards = passes * world
        my_shards = [rank * passes + q for q in range(passes)]
        rank_accs = []
        if rehearsal:  # shard I of S (S doubled with passes if it does not fit)
            shards = args.rehearse_shards * (passes // max(1, -(-wl["fit_shards"] // world)))
            my_shards = [args.rehearse_index] if args.rehearse_index >= 0 else list(range(shards))
            if any(s >= shards for s in my_shards):
                raise SystemExit(f"--rehearse-index {args.rehearse_index}: only {shards} shards")
        err = None
        try:
            if rehearsal:  # one engine per rehearsed rank, in sequence (each its own timed window)
                for s in my_shards:
                    rank_accs.append(run_shards(args, wl, topo, ev, [s], shards, dist, dev, local, rank,
                                                flags | shard_flags(shard_rule(shards), args.fresh_tiles)))
                acc = max(rank_accs, key=lambda a: a["elapsed"])  # the job waits for its slowest rank
            else:
                acc = run_shards(args, wl, topo, ev, my_shards, shards, dist, dev, local, rank,
                                 flags | shard_flags(shard_rule(shards), args.fresh_tiles))
        except gossip.GossipError as e:
            if getattr(e, "code", None) not in CAPACITY_CODES:
                raise
            err = e
        failed = 1.0 if err else 0.0
        if dist:
            failed = gd.allreduce_scalars([failed], op="max", device=dev)[0]
        if not failed:
            break
        if rank == 0:
            log(f"[bench] {shards} shards do not fit ({err or 'another rank'}): retrying with {2 * shards}")
        retried.append(shards)
        passes *= 2
    layout = (f"{shards} share shards, {len(my_shards)} per GPU in sequence" if len(my_shards) > 1
              else f"{shards} share shards, one per GPU")
    if rehearsal:
        which = (f"shard {my_shards[0]}" if len(my_shards) == 1 else
                 f"shards 0..{shards - 1} one after another, the slowest one's window")
        wl["desc"] += f" [REHEARSAL: {which} of {shards} on one GPU]"
        layout = f"{shards} share shards, one per GPU"

    elapsed, edges, pull_ms = acc["elapsed"], acc["edges"], acc["pull_ms"]
    launches = acc["launches"]
    if dist:
        elapsed, pull_ms_max = gd.allreduce_scalars([elapsed, pull_ms], op="max", device=dev)
        edges_total, gens_total = gd.allreduce_scalars([edges, acc["gens"]], op="sum", device=dev)
        edges_total = int(edges_total)
    else:
        edges_total, gens_total, pull_ms_max = edges, acc["gens"], pull_ms
    if not rehearsal:
        # every counted generation of the simulated ticks ran on exactly one shard
        want = int(np.count_nonzero(ev["ns"] < (SLICE_NS // L_NS + W + K) * L_NS))
        if int(gens_total) != want:
            raise SystemExit(f"shard coverage broken: {int(gens_total)} generations vs {want}")

    if rank == 0:
        avg_ms = pull_ms / max(launches, 1)
        # Algorithmic bytes per launch of the implemented pull: 16 B per
        # (edge, word-pair) neighbour read actually needed + 4 B per peer id + 8 B per peer
        # occupancy word + 16 B per own-row seen/F access + per-node row_ptr/counters/occupancy.
        per_launch = lambda x: float(x) / max(launches, 1)  # noqa: E731
        bytes_per_launch = per_launch(acc["moved"])
        dense_bytes_per_launch = per_launch(acc["dense"])  # SURVEY §8d dense formula
        achieved = bytes_per_launch / (avg_ms * 1e6) if avg_ms > 0 else 0.0  # GB/s
        tick0 = SLICE_NS // L_NS
        out = {
            "metric": (BASELINE_METRIC if wl["name"] == "C4" and not rehearsal and "GOSSIP_BENCH_NODES" not in os.environ
                       else "share-deliveries/sec (edge events)"),
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
                "workload": f"{wl['desc']}, {n_gpus} GPU(s), {layout}",
                "nodes": n,
                "avg_degree": 16,
                "latency_ms": 5,
                "ticks_timed": [tick0 + W, tick0 + W + K],
                "ramp_ticks_before_timing": acc["ramp_ticks"],
                "slice_schedule": sinfo,
                "edge_events_timed": edges_total,
                "share_shards": shards,
                "shards_retried": retried,
                "shards_per_gpu": len(my_shards),
                "live_words_per_node": acc["words_hw"],
                "window_capacity_words": acc["words_cap"],
                "window_early_retires": acc.get("early_retires", 0),
                "device_gib": acc["dev_bytes"] / 2**30,
                "parallelism": f"share-shard x{shards} over {max(world, 1)} rank(s)",
                "shard_rule": shard_rule(shards),
                "fresh_tile_per_tick": bool(shard_flags(shard_rule(shards), args.fresh_tiles) & gossip.F_TILE_PER_TICK),
            },
            "roofline": None,
        }
        if rehearsal:
            out["config"]["rehearsed_shards"] = my_shards
            if len(rank_accs) > 1:  # every rank's timed window: ms per tick, window peak, edges
                out["config"]["rank_ms_per_step"] = [a["elapsed"] * 1e3 / K for a in rank_accs]
                out["config"]["rank_live_words"] = [a["words_hw"] for a in rank_accs]
                out["config"]["rank_window_capacity_words"] = [a["words_cap"] for a in rank_accs]
                out["config"]["rank_edge_events"] = [a["edges"] for a in rank_accs]
                out["config"]["rank_phase_ms_per_tick"] = [a["phase_ms"] / max(a["launches"], 1) for a in rank_accs]
                out["config"]["edge_events_all_ranks"] = int(sum(a["edges"] for a in rank_accs))
                # what an S-GPU job of these ranks would reach (unmeasured on an S-GPU node): every
                # rank's edge events over the slowest rank's window
                out["config"]["projected_job_value"] = out["config"]["edge_events_all_ranks"] / elapsed
        k_pull = {
            "kernel": "k_pull",
            "avg_launch_ms": avg_ms,
            "launches": launches,
            "bytes_per_launch": bytes_per_launch,
            "achieved": achieved,
            "frac": achieved / HBM_PEAK_GBS,
            "bytes_note": "algorithmic bytes of the occupancy-skipping pull: the peer-row, peer-id, "
                          "occupancy, own-row and counter bytes it must move",
            "dense_formula_bytes_per_launch": dense_bytes_per_launch,
            "dense_formula_frac": ((dense_bytes_per_launch / (avg_ms * 1e6)) / HBM_PEAK_GBS) if avg_ms > 0 else None,
            "dense_formula_note": "SURVEY 8(d) B = 8(n+1)+4nnz+8Wq*nnz+24Wq*n+16n assumes every "
                                  "peer-row word is read; the kernel skips dead, saturated and "
                                  "unoccupied rows, so this ratio can exceed 1 and is not a "
                                  "roofline fraction",
            "bytes_breakdown_per_launch": {
                "peer_rows": per_launch(16 * acc["pe"]),
                "peer_ids": per_launch(4 * acc["col"]),
                "peer_occupancy": per_launch(8 * acc["nz"]),
                "own_seen_read": per_launch(16 * acc["srd"]),
                "own_seen_write": per_launch(16 * acc["swr"]),
                "frontier_write": per_launch(16 * acc["fwr"]),
                "per_node_rowptr_counters_occupancy_sat": per_launch(
                    acc["moved"] - 16 * acc["pe"] - 4 * acc["col"] - 8 * acc["nz"] -
                    16 * (acc["srd"] + acc["swr"] + acc["fwr"])),
            },
            "breakdown_sums_to_bytes": True,  # (the last item is the remainder of the engine's count)
            "saturated_tiles_skipped_per_launch": per_launch(acc.get("sat_skips", 0)),
            "items_per_launch": per_launch(acc.get("items", 0)),
            "gather_items_per_launch": per_launch(acc.get("gather_items", 0)),
            "dense_row_tiles_last_tick": acc.get("dense_tiles", 0),
        }
        opts = acc.get("options", {})
        overlap = opts.get("young_overlap", 1)
        variant = {"nt_rows": acc["nt"], "grid": acc["grid"],
                   "young_overlap": overlap if acc["young_launches"] else None,
                   "late_age": acc.get("late_age", 0), "pull_tiles": acc.get("pull_tiles", 0),
                   "lanes_per_node": acc.get("lpw", 0), "pull_sat": acc.get("pull_sat", 0),
                   "dense_rows": 1 if acc.get("dense_tiles", 0) else 0,
                   "young_grid_blocks": acc.get("young_grid", 0) if acc["young_launches"] else None,
                   "options": opts, "lib_sha256": lib_build_id()}
        t_pull, why_pull = pmc_traffic(wl["name"], out, variant)
        k_pull["traffic"] = t_pull
        young = None
        if acc["young_launches"]:
            yl = acc["young_launches"]
            y_ms = acc["young_ms"] / yl
            ybd = young_breakdown(acc, yl, n)
            young = {
                "kernel": "k_pull_young",
                "avg_launch_ms": y_ms,
                "launches": yl,
                "bytes_per_launch": acc["young_bytes"] / yl,
                "achieved": acc["young_bytes"] / yl / (y_ms * 1e6) if y_ms > 0 else None,
                "slot_lines_per_launch": acc["young_sl"] / yl,
                "fallback_rows_per_launch": acc["young_fb"] / yl,
                "second_lines_unhinted_per_launch": acc.get("young_line2_misses", 0) / yl,
                "bytes_breakdown_per_launch": ybd,
                "breakdown_sums_to_bytes": abs(sum(ybd.values()) - acc["young_bytes"] / yl) <= 1e-6 * acc["young_bytes"] / yl,
            }
            t_young, why_young = pmc_traffic(wl["name"] + "_young", out, variant)
            young["traffic"] = t_young
        if young is None:
            roof = dict(k_pull)
            roof.update({"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "pull_variant": variant})
            if why_pull:
                roof["traffic_note"] = why_pull
        else:
            # The pull phase: k_pull and k_pull_young, concurrent on two streams (young_overlap),
            # timed as one unit by HIP events around both on the engine stream.  Its bytes are
            # the two kernels' algorithmic bytes, its traffic the sum of their PMC passes.
            ph_ms = (acc["phase_ms"] / max(launches, 1)) if acc["phase_ms"] else \
                avg_ms + acc["young_ms"] / max(launches, 1)
            ph_b = bytes_per_launch + young["bytes_per_launch"]
            ph_ach = ph_b / (ph_ms * 1e6) if ph_ms > 0 else 0.0
            traffic = (t_pull + t_young) if (t_pull is not None and t_young is not None) else None
            roof = {
                "bound": "hbm",
                "achieved": ph_ach,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": ph_ach / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": "pull phase: k_pull + k_pull_young" +
                          (" (concurrent, two streams)" if overlap else " (in sequence)"),
                # what `frac` is a fraction of: the bytes the skipping pull must move,
                # itemised per kernel below; SURVEY 8(d)'s dense formula, which assumes every peer-row
                # word is read, gives the second ratio (> 1: the kernels skip most of those rows)
                "frac_basis": "achieved = algorithmic bytes of the skipping pull (k_pull's peer rows, "
                              "ids, occupancy, own rows, counters + k_pull_young's slot lines, lists, rows) "
                              "/ phase time; peak = 8 TB/s",
                "dense_formula_frac": ((dense_bytes_per_launch / (ph_ms * 1e6)) / HBM_PEAK_GBS) if ph_ms > 0 else None,
                "avg_launch_ms": ph_ms,
                "launches": launches,
                "bytes_per_launch": ph_b,
                "pull_variant": variant,
                "kernels": {"k_pull": k_pull, "k_pull_young": young},
            }
            why = "; ".join(w for w in (why_pull, why_young) if w)
            if why:
                roof["traffic_note"] = why
        roof["pull_fraction_of_step"] = ((roof["avg_launch_ms"] * launches / 1e3) / elapsed) if elapsed > 0 else None
        out["roofline"] = roof
        if n_gpus == 1 and world == 1 and not args.no_cpu_baseline:
            try:
                win = ev[ev["ns"] >= SLICE_NS]
                out["cpu_baseline"] = cpu_baseline(topo, win, args.cpu_sample, args.cpu_hops)
            except Exception as e:  # the baseline is reported, never required
                out["cpu_baseline"] = {"value": None, "error": str(e)}
            try:
                win = ev[ev["ns"] >= SLICE_NS]
                out["cpu_baseline_bitsliced"] = cpu_baseline_bitsliced(topo, win, 64, args.cpu_hops,
                                                                       args.threads)
            except Exception as e:
                out["cpu_baseline_bitsliced"] = {"value": None, "error": str(e)}
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
