"""Python host mirror of the MI355X gossip engine (ctypes over libgossip.so's C ABI).

The product's host side is C++ (``csrc/gossip_sim.cpp``, like the reference's
``p2pnetwork.cc``); this module is the thin binding that tests and ``bench.py`` use.  It
mirrors the reference's ``P2PGossipNetworkSimulation`` (p2pnetwork.cc:15-286) so parity
tests read like the reference's own program:

    sim = P2PGossipNetworkSimulation(numNodes)          # p2pnetwork.cc:40-50
    sim.CreateRandomTopology(connectionProbability, latency)   # :62-96
    sim.Start(simulationTime)                           # :193-218
    sim.PrintStatistics()                               # :253-285

There is no CPU fallback: every call goes through ``libgossip.so`` and the engine refuses to
start without a HIP device.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(os.path.dirname(_HERE), "lib")
LIB_PATH = os.environ.get("GOSSIP_LIB_PATH") or os.path.join(LIB_DIR, "libgossip.so")

TOPO_EXACT = 0
TOPO_SKIP = 1
MODE_AUTO = 0
MODE_CSR = 1
MODE_DENSE = 2
F_TRACE = 1
F_TIMING = 2
F_NOSKIP = 4
F_TILE_PER_TICK = 32
F_HANDSHAKE = 64
F_HOP_BATCH = 128
F_SHARD_BY_TICK = 256

EXPORTED_SYMBOLS = (
    "gossip_last_error", "gossip_version", "gossip_seconds_to_ns", "gossip_milliseconds_to_ns",
    "gossip_topology_create", "gossip_topology_from_links", "gossip_topology_num_nodes",
    "gossip_topology_num_links", "gossip_topology_get_links", "gossip_topology_num_entries",
    "gossip_topology_get_csr", "gossip_topology_get_degrees", "gossip_topology_destroy",
    "gossip_schedule_create", "gossip_schedule_from_events", "gossip_schedule_size",
    "gossip_schedule_get", "gossip_schedule_destroy", "gossip_shard_events", "gossip_shard_events_by_tick",
    "gossip_engine_create", "gossip_engine_set_graph", "gossip_engine_set_topology",
    "gossip_engine_set_schedule", "gossip_engine_set_schedule_obj", "gossip_engine_add_snapshot",
    "gossip_engine_first_tick", "gossip_engine_end_tick", "gossip_engine_current_tick",
    "gossip_engine_run", "gossip_engine_sync", "gossip_engine_get_stats",
    "gossip_engine_get_snapshot", "gossip_engine_get_counters", "gossip_engine_reset_timing",
    "gossip_engine_trace_size", "gossip_engine_get_trace", "gossip_engine_destroy",
    "gossip_format_statistics", "gossip_format_periodic", "gossip_engine_set_link_timing",
    "gossip_share_message_length", "gossip_format_event_log", "gossip_engine_set_row_partition",
    "gossip_rccl_unique_id", "gossip_engine_connect_rccl", "gossip_engine_group_run",
    "gossip_engine_set_option", "gossip_engine_mode", "gossip_engine_tick_begin",
    "gossip_engine_exchange_export", "gossip_engine_exchange_import", "gossip_engine_tick_end",
    "gossip_schedule_create_philox", "gossip_engine_exchange_chunks",
    "gossip_engine_exchange_export_chunk", "gossip_engine_exchange_import_chunk",
    "gossip_format_netanim", "gossip_topology_load_links", "gossip_schedule_load_events",
    "gossip_engine_abort", "gossip_engine_get_rehearsal", "gossip_engine_get_rehearsal_peak",
    "gossip_engine_get_option",
)

# NS-3 5 Mbps point-to-point links (p2pnetwork.cc:113): ns per byte, PPP+IPv4+TCP(timestamp
# option) header bytes, TcpSocketBase's one-TimeStep send deferral (gossip.h)
LINK_5MBPS = (1600, 54, 1)

GEN_EVENT_DTYPE = np.dtype([("ns", "<i8"), ("node", "<u4"), ("share_id", "<u4")])


class GossipError(RuntimeError):
    """A failed C-ABI call; ``code`` is the GOSSIP_E* status (gossip.h)."""

    def __init__(self, msg: str, code: int = 0):
        super().__init__(msg)
        self.code = code


E_INVAL, E_HIP, E_NOMEM, E_STATE, E_CAPACITY = -1, -2, -3, -4, -5


class gossip_config(C.Structure):
    _fields_ = [
        ("num_nodes", C.c_uint32), ("latency_ns", C.c_int64), ("t_start_ns", C.c_int64),
        ("t_cut_ns", C.c_int64), ("device", C.c_int32), ("mode", C.c_int32),
        ("max_words", C.c_uint32), ("shard_rank", C.c_uint32), ("shard_count", C.c_uint32),
        ("flags", C.c_uint32),
    ]


class gossip_counters(C.Structure):
    _fields_ = [
        ("edge_events", C.c_uint64), ("receptions", C.c_uint64), ("generations", C.c_uint64),
        ("ticks", C.c_uint64), ("pull_launches", C.c_uint64), ("pull_ms", C.c_double),
        ("pull_bytes", C.c_uint64), ("words_hw", C.c_uint32), ("words_cap", C.c_uint32),
        ("device_bytes", C.c_uint64), ("pull_bytes_moved", C.c_uint64),
        ("pull_pair_edges", C.c_uint64), ("dense_ops", C.c_uint64),
        ("dense_tiles_skipped", C.c_uint64), ("pull_col_ids", C.c_uint64),
        ("pull_seen_reads", C.c_uint64), ("pull_seen_writes", C.c_uint64),
        ("pull_f_writes", C.c_uint64), ("pull_nz_reads", C.c_uint64),
        ("pull_nt", C.c_uint32), ("pull_grid", C.c_uint32),
        ("young_ms", C.c_double), ("young_launches", C.c_uint64),
        ("young_bytes_moved", C.c_uint64), ("young_slot_lines", C.c_uint64),
        ("young_col_ids", C.c_uint64), ("young_fallback_rows", C.c_uint64),
        ("young_seen_reads", C.c_uint64), ("young_seen_writes", C.c_uint64),
        ("young_rows_written", C.c_uint64), ("young_slot_writes", C.c_uint64),
        ("exchange_bytes_sent", C.c_uint64), ("exchange_bytes_received", C.c_uint64),
        ("pull_phase_ms", C.c_double), ("young_line2_misses", C.c_uint64),
        ("pull_late_age", C.c_uint32), ("pull_tiles", C.c_uint32),
        ("young_fresh_lines", C.c_uint64),
        ("pull_lpw", C.c_uint32), ("pull_dense_tiles", C.c_uint32),
        ("pull_sat_skips", C.c_uint64), ("pull_sat", C.c_uint32), ("pad0", C.c_uint32),
        ("window_early_retires", C.c_uint64), ("young_list_lines", C.c_uint64),
        ("pull_items", C.c_uint64), ("pull_gather_items", C.c_uint64),
        ("dense_fused_launches", C.c_uint64),
        ("young_grid", C.c_uint32), ("young_skip_ticks", C.c_uint32),
        ("pull_push_tiles", C.c_uint64), ("pull_pushw_tiles", C.c_uint64), ("pull_marks", C.c_uint64),
        ("young_idle_ticks", C.c_uint64),
    ]


_lib = None


def _ptr(a, ct):
    return a.ctypes.data_as(C.POINTER(ct)) if a is not None else None


def load_library(path: str = LIB_PATH):
    """Load libgossip.so (build it with ``__graft_entry__.build()``); raise if missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise GossipError(f"{path} not built: run __graft_entry__.build() (no CPU fallback)")
    lib = C.CDLL(path)
    P, u32, u64, i64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int64, C.c_int32
    sig = {
        "gossip_last_error": (C.c_char_p, []),
        "gossip_version": (C.c_char_p, []),
        "gossip_seconds_to_ns": (i64, [C.c_double]),
        "gossip_milliseconds_to_ns": (i64, [C.c_double]),
        "gossip_topology_create": (C.c_int, [u32, C.c_double, u32, C.c_int, C.c_int, C.POINTER(P)]),
        "gossip_topology_from_links": (C.c_int, [u32, u64, P, P, C.POINTER(P)]),
        "gossip_topology_load_links": (C.c_int, [u32, C.c_char_p, C.POINTER(P)]),
        "gossip_schedule_load_events": (C.c_int, [u32, C.c_char_p, C.POINTER(P)]),
        "gossip_engine_abort": (C.c_int, [P]),
        "gossip_engine_get_rehearsal": (C.c_int, [P, u32, P, P, P, P, C.POINTER(u64)]),
        "gossip_engine_get_rehearsal_peak": (C.c_int, [P, u32, P]),
        "gossip_engine_get_option": (C.c_int, [P, C.c_char_p, C.POINTER(i64)]),
        "gossip_topology_num_nodes": (u32, [P]),
        "gossip_topology_num_links": (u64, [P]),
        "gossip_topology_get_links": (C.c_int, [P, P, P]),
        "gossip_topology_num_entries": (u64, [P]),
        "gossip_topology_get_csr": (C.c_int, [P, P, P, P]),
        "gossip_topology_get_degrees": (C.c_int, [P, P, P]),
        "gossip_topology_destroy": (None, [P]),
        "gossip_schedule_create": (C.c_int, [u32, u32, i64, i64, i64, u32, C.c_int, C.POINTER(P)]),
        "gossip_schedule_from_events": (C.c_int, [u64, P, C.POINTER(P)]),
        "gossip_schedule_create_philox": (C.c_int, [u32, u32, i64, i64, i64, i32, C.POINTER(P)]),
        "gossip_schedule_size": (u64, [P]),
        "gossip_schedule_get": (C.c_int, [P, P]),
        "gossip_schedule_destroy": (None, [P]),
        "gossip_shard_events": (C.c_int, [P, u64, P, u32, P]),
        "gossip_shard_events_by_tick": (C.c_int, [P, u64, P, u32, i64, P]),
        "gossip_engine_create": (C.c_int, [C.POINTER(gossip_config), C.POINTER(P)]),
        "gossip_engine_set_graph": (C.c_int, [P, u32, P, P, P]),
        "gossip_engine_set_topology": (C.c_int, [P, P]),
        "gossip_engine_set_schedule": (C.c_int, [P, u64, P]),
        "gossip_engine_set_schedule_obj": (C.c_int, [P, P]),
        "gossip_engine_add_snapshot": (C.c_int, [P, i64]),
        "gossip_engine_set_link_timing": (C.c_int, [P, i64, u32, i64]),
        "gossip_share_message_length": (u32, [u32, u32, i64]),
        "gossip_engine_set_row_partition": (C.c_int, [P, u32, u32]),
        "gossip_rccl_unique_id": (C.c_int, [C.c_char_p, u32]),
        "gossip_engine_connect_rccl": (C.c_int, [P, C.c_char_p, u32]),
        "gossip_engine_group_run": (C.c_int, [P, u32, i64]),
        "gossip_engine_set_option": (C.c_int, [P, C.c_char_p, i64]),
        "gossip_engine_mode": (C.c_int, [P]),
        "gossip_engine_tick_begin": (C.c_int, [P]),
        "gossip_engine_exchange_export": (C.c_int, [P, P, u64, C.POINTER(u64)]),
        "gossip_engine_exchange_import": (C.c_int, [P, u32, P, u64]),
        "gossip_engine_tick_end": (C.c_int, [P]),
        "gossip_engine_exchange_chunks": (C.c_int, [P]),
        "gossip_engine_exchange_export_chunk": (C.c_int, [P, u32, P, u64, C.POINTER(u64)]),
        "gossip_engine_exchange_import_chunk": (C.c_int, [P, u32, u32, P, u64]),
        "gossip_format_netanim": (i64, [P, u64, P, u64, P, P, P, i64, i64, i64, u32, i64, C.c_int,
                                        C.c_char_p, u64]),
        "gossip_format_event_log": (i64, [P, u64, P, u64, P, P, P, P, i64, i64, i64, i64, u32,
                                          i64, C.c_int, C.c_char_p, u64]),
        "gossip_engine_first_tick": (i64, [P]),
        "gossip_engine_end_tick": (i64, [P]),
        "gossip_engine_current_tick": (i64, [P]),
        "gossip_engine_run": (C.c_int, [P, i64]),
        "gossip_engine_sync": (C.c_int, [P]),
        "gossip_engine_get_stats": (C.c_int, [P, P, P, P, P, P, P, P]),
        "gossip_engine_get_snapshot": (C.c_int, [P, u32, P, P, P]),
        "gossip_engine_get_counters": (C.c_int, [P, C.POINTER(gossip_counters)]),
        "gossip_engine_reset_timing": (C.c_int, [P]),
        "gossip_engine_trace_size": (u64, [P]),
        "gossip_engine_get_trace": (C.c_int, [P, P, P, P, P, P]),
        "gossip_engine_destroy": (None, [P]),
        "gossip_format_statistics": (i64, [u32, P, P, P, P, P, P, P, C.c_char_p, u64]),
        "gossip_format_periodic": (i64, [C.c_double, u32, u64, u64, u64, C.c_char_p, u64]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _check(rc: int, what: str):
    if rc != 0:
        raise GossipError(f"{what}: {load_library().gossip_last_error().decode()} (code {rc})", rc)


def _vp(a):
    return C.c_void_p(a.ctypes.data) if a is not None and a.size else None


def rccl_unique_id() -> bytes:
    """An RCCL communicator id (128 bytes) to share with every rank of a row partition."""
    buf = C.create_string_buffer(128)
    _check(load_library().gossip_rccl_unique_id(buf, 128), "rccl unique id")
    return buf.raw


def group_run(engines, tick_end: int | None = None):
    """Step the engines of one row partition (ranks 0..count-1, one device) in lockstep."""
    arr = (C.c_void_p * len(engines))(*[e._h.value if hasattr(e._h, "value") else e._h for e in engines])
    end = engines[0].end_tick if tick_end is None else int(tick_end)
    _check(load_library().gossip_engine_group_run(arr, len(engines), end), "group run")


def share_message_length(origin: int, share_id: int, t_ns: int) -> int:
    """len(Share::ToString()) of a share generated at t_ns (p2pnode.cc:6-11)."""
    return int(load_library().gossip_share_message_length(int(origin), int(share_id), int(t_ns)))


def seconds_to_ns(s: float) -> int:
    return int(load_library().gossip_seconds_to_ns(float(s)))


def milliseconds_to_ns(ms: float) -> int:
    return int(load_library().gossip_milliseconds_to_ns(float(ms)))


class Topology:
    """G(n,p) link set with the reference's fix-up (p2pnetwork.cc:62-96) and its peer lists."""

    def __init__(self, handle):
        self._h = C.c_void_p(handle)

    @classmethod
    def gnp(cls, n: int, p: float, seed: int, kind: int = TOPO_EXACT, threads: int = 8):
        lib = load_library()
        h = C.c_void_p()
        _check(lib.gossip_topology_create(n, p, seed, kind, threads, C.byref(h)), "topology")
        return cls(h.value)

    @classmethod
    def from_links(cls, n: int, a, b):
        lib = load_library()
        a = np.ascontiguousarray(a, dtype=np.uint32)
        b = np.ascontiguousarray(b, dtype=np.uint32)
        h = C.c_void_p()
        _check(lib.gossip_topology_from_links(n, a.size, _vp(a), _vp(b), C.byref(h)), "topology")
        return cls(h.value)

    @classmethod
    def load_links(cls, n: int, path: str):
        """A key list written by gossip_sim --dumpLinks, parsed strictly (GossipError, code
        GOSSIP_EINVAL, naming the line of any malformed entry)."""
        lib = load_library()
        h = C.c_void_p()
        _check(lib.gossip_topology_load_links(n, os.fsencode(path), C.byref(h)), "load links")
        return cls(h.value)

    @property
    def num_nodes(self) -> int:
        return int(load_library().gossip_topology_num_nodes(self._h))

    def links(self):
        lib = load_library()
        m = int(lib.gossip_topology_num_links(self._h))
        a = np.empty(m, np.uint32)
        b = np.empty(m, np.uint32)
        _check(lib.gossip_topology_get_links(self._h, _vp(a), _vp(b)), "links")
        return a, b

    def csr(self):
        lib = load_library()
        n = self.num_nodes
        nnz = int(lib.gossip_topology_num_entries(self._h))
        rp = np.empty(n + 1, np.int64)
        col = np.empty(nnz, np.int32)
        mult = np.empty(nnz, np.uint8)
        _check(lib.gossip_topology_get_csr(self._h, _vp(rp), _vp(col), _vp(mult)), "csr")
        return rp, col, mult

    def degrees(self):
        lib = load_library()
        n = self.num_nodes
        peers = np.empty(n, np.uint32)
        sockets = np.empty(n, np.uint32)
        _check(lib.gossip_topology_get_degrees(self._h, _vp(peers), _vp(sockets)), "degrees")
        return peers, sockets

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.gossip_topology_destroy(self._h)
            self._h = None


def make_schedule(n: int, node_seed: int, t_start_ns: int, t_cut_ns: int, t_gen_end_ns: int = 0,
                  id_mask: int = 0, threads: int = 8) -> np.ndarray:
    """Counted share generations (p2pnode.cc:91-125, 201-209) as a GEN_EVENT_DTYPE array."""
    lib = load_library()
    h = C.c_void_p()
    _check(lib.gossip_schedule_create(n, node_seed, t_start_ns, t_cut_ns, t_gen_end_ns, id_mask,
                                      threads, C.byref(h)), "schedule")
    try:
        m = int(lib.gossip_schedule_size(h))
        ev = np.empty(m, GEN_EVENT_DTYPE)
        if m:
            _check(lib.gossip_schedule_get(h, _vp(ev)), "schedule get")
        return ev
    finally:
        lib.gossip_schedule_destroy(h)


def load_events(n: int, path: str) -> np.ndarray:
    """Generation events written by gossip_sim --dumpEvents ("ns node shareId" per line), parsed
    strictly like Topology.load_links; sorted by (ns, node)."""
    lib = load_library()
    h = C.c_void_p()
    _check(lib.gossip_schedule_load_events(n, os.fsencode(path), C.byref(h)), "load events")
    try:
        m = int(lib.gossip_schedule_size(h))
        ev = np.empty(m, GEN_EVENT_DTYPE)
        if m:
            _check(lib.gossip_schedule_get(h, _vp(ev)), "schedule get")
        return ev
    finally:
        lib.gossip_schedule_destroy(h)


def make_schedule_philox(n: int, seed: int, t_start_ns: int, t_cut_ns: int, t_gen_end_ns: int = 0,
                         device: int = 0) -> np.ndarray:
    """Synthetic schedule generated on the GPU from per-node Philox4x32-10 streams (gossip.h
    gossip_schedule_create_philox): the reference's rules, not its mt19937 stream."""
    lib = load_library()
    h = C.c_void_p()
    _check(lib.gossip_schedule_create_philox(n, seed, t_start_ns, t_cut_ns, t_gen_end_ns, device,
                                             C.byref(h)), "philox schedule")
    try:
        m = int(lib.gossip_schedule_size(h))
        ev = np.empty(m, GEN_EVENT_DTYPE)
        if m:
            _check(lib.gossip_schedule_get(h, _vp(ev)), "schedule get")
        return ev
    finally:
        lib.gossip_schedule_destroy(h)


def shard_events(topo: "Topology", ev: np.ndarray, shard_count: int, by_tick_latency_ns: int = 0) -> np.ndarray:
    """Owner shard of every generation event (the engines' multi-GPU sharding rule): the hash rule,
    or with by_tick_latency_ns > 0 the birth-tick rule of GOSSIP_F_SHARD_BY_TICK."""
    ev = np.ascontiguousarray(ev, GEN_EVENT_DTYPE)
    owner = np.empty(ev.size, np.uint32)
    lib = load_library()
    if by_tick_latency_ns > 0:
        rc = lib.gossip_shard_events_by_tick(topo._h, ev.size, _vp(ev), shard_count, int(by_tick_latency_ns), _vp(owner))
    else:
        rc = lib.gossip_shard_events(topo._h, ev.size, _vp(ev), shard_count, _vp(owner))
    _check(rc, "shard events")
    return owner


def events_from_arrays(ns, node, share_id) -> np.ndarray:
    ev = np.empty(len(ns), GEN_EVENT_DTYPE)
    ev["ns"] = ns
    ev["node"] = node
    ev["share_id"] = share_id
    return ev


@dataclass
class Stats:
    gen: np.ndarray
    recv: np.ndarray
    fwd: np.ndarray
    sent: np.ndarray
    processed: np.ndarray
    peers: np.ndarray
    sockets: np.ndarray


class Engine:
    """The tick-synchronous HIP engine (one tick = Latency)."""

    def __init__(self, num_nodes: int, latency_ns: int, t_start_ns: int, t_cut_ns: int,
                 device: int = 0, mode: int = MODE_AUTO, max_words: int = 0, shard_rank: int = 0,
                 shard_count: int = 1, flags: int = 0):
        lib = load_library()
        cfg = gossip_config(num_nodes, latency_ns, t_start_ns, t_cut_ns, device, mode, max_words,
                            shard_rank, shard_count, flags)
        h = C.c_void_p()
        _check(lib.gossip_engine_create(C.byref(cfg), C.byref(h)), "engine create")
        self._h = h
        self.n = num_nodes

    def set_topology(self, topo: Topology):
        _check(load_library().gossip_engine_set_topology(self._h, topo._h), "set topology")

    def set_graph(self, row_ptr, col, mult=None):
        row_ptr = np.ascontiguousarray(row_ptr, np.int64)
        col = np.ascontiguousarray(col, np.int32)
        mult = None if mult is None else np.ascontiguousarray(mult, np.uint8)
        _check(load_library().gossip_engine_set_graph(self._h, self.n, _vp(row_ptr), _vp(col),
                                                      _vp(mult)), "set graph")

    def add_snapshot(self, t_ns: int):
        _check(load_library().gossip_engine_add_snapshot(self._h, int(t_ns)), "snapshot")

    def set_row_partition(self, rank: int, count: int):
        """Own node rows [rank block] only; exchange via connect_rccl or group_run (gossip.h)."""
        _check(load_library().gossip_engine_set_row_partition(self._h, int(rank), int(count)),
               "row partition")

    def set_option(self, name: str, value: int):
        """Tuning option (gossip.h gossip_engine_set_option): pull_nt, pull_grid, young, ...,
        dense_fused.  Results never depend on them."""
        _check(load_library().gossip_engine_set_option(self._h, name.encode(), int(value)),
               f"option {name}")

    def get_option(self, name: str) -> int:
        """The value option `name` holds (gossip_engine_get_option)."""
        v = C.c_int64()
        _check(load_library().gossip_engine_get_option(self._h, name.encode(), C.byref(v)), f"option {name}")
        return int(v.value)

    def connect_rccl(self, unique_id: bytes):
        _check(load_library().gossip_engine_connect_rccl(self._h, unique_id, len(unique_id)),
               "rccl connect")

    def abort(self):
        """gossip_engine_abort: tear down the communicator (if any); later steps fail (E_STATE)."""
        _check(load_library().gossip_engine_abort(self._h), "abort")

    # ---- host-staged row exchange (gossip.h): one message per rank and tick, or per row chunk --
    def tick_begin(self) -> bool:
        """Enqueue pull + births of the next tick (row chunk by row chunk); False when done."""
        rc = load_library().gossip_engine_tick_begin(self._h)
        if rc == 1:
            return False
        _check(rc, "tick begin")
        return True

    def exchange_export(self) -> np.ndarray:
        lib = load_library()
        n = C.c_uint64()
        _check(lib.gossip_engine_exchange_export(self._h, None, 0, C.byref(n)), "export size")
        buf = np.empty(n.value // 8, np.uint64)
        _check(lib.gossip_engine_exchange_export(self._h, _vp(buf), buf.nbytes, C.byref(n)), "export")
        return buf

    def exchange_import(self, rank: int, msg: np.ndarray):
        msg = np.ascontiguousarray(msg, np.uint64)
        _check(load_library().gossip_engine_exchange_import(self._h, int(rank), _vp(msg), msg.nbytes),
               "import")

    def exchange_chunks(self) -> int:
        """Row chunks of the pipelined exchange (option xchunks; 1 without a row partition)."""
        rc = load_library().gossip_engine_exchange_chunks(self._h)
        _check(min(rc, 0), "exchange chunks")
        return rc

    def exchange_export_chunk(self, chunk: int) -> np.ndarray:
        """This rank's message of row chunk `chunk` (waits for that chunk only)."""
        lib = load_library()
        n = C.c_uint64()
        _check(lib.gossip_engine_exchange_export_chunk(self._h, int(chunk), None, 0, C.byref(n)), "export size")
        buf = np.empty(n.value // 8, np.uint64)
        _check(lib.gossip_engine_exchange_export_chunk(self._h, int(chunk), _vp(buf), buf.nbytes, C.byref(n)),
               "export")
        return buf

    def exchange_import_chunk(self, rank: int, chunk: int, msg: np.ndarray):
        msg = np.ascontiguousarray(msg, np.uint64)
        _check(load_library().gossip_engine_exchange_import_chunk(self._h, int(rank), int(chunk), _vp(msg),
                                                                   msg.nbytes), "import")

    def tick_end(self):
        _check(load_library().gossip_engine_tick_end(self._h), "tick end")

    def set_link_timing(self, ns_per_byte: int, header_bytes: int, send_defer_ns: int):
        _check(load_library().gossip_engine_set_link_timing(
            self._h, int(ns_per_byte), int(header_bytes), int(send_defer_ns)), "link timing")

    def set_schedule(self, ev: np.ndarray):
        ev = np.ascontiguousarray(ev, GEN_EVENT_DTYPE)
        _check(load_library().gossip_engine_set_schedule(self._h, ev.size, _vp(ev)), "set schedule")

    @property
    def mode(self) -> int:
        """MODE_CSR or MODE_DENSE (MODE_AUTO resolves when the graph is set)."""
        return int(load_library().gossip_engine_mode(self._h))

    @property
    def first_tick(self) -> int:
        return int(load_library().gossip_engine_first_tick(self._h))

    @property
    def end_tick(self) -> int:
        return int(load_library().gossip_engine_end_tick(self._h))

    @property
    def current_tick(self) -> int:
        return int(load_library().gossip_engine_current_tick(self._h))

    def run(self, tick_end: int | None = None):
        if tick_end is None:
            tick_end = self.end_tick
        _check(load_library().gossip_engine_run(self._h, int(tick_end)), "run")

    def sync(self):
        _check(load_library().gossip_engine_sync(self._h), "sync")

    def stats(self) -> Stats:
        n = self.n
        a = [np.empty(n, np.uint32) for _ in range(3)]
        sent = np.empty(n, np.uint64)
        b = [np.empty(n, np.uint32) for _ in range(3)]
        _check(load_library().gossip_engine_get_stats(self._h, _vp(a[0]), _vp(a[1]), _vp(a[2]),
                                                      _vp(sent), _vp(b[0]), _vp(b[1]), _vp(b[2])),
               "stats")
        return Stats(a[0], a[1], a[2], sent, b[0], b[1], b[2])

    def snapshot(self, k: int):
        t = C.c_int64()
        g = C.c_uint64()
        p = C.c_uint64()
        _check(load_library().gossip_engine_get_snapshot(self._h, k, C.byref(t), C.byref(g),
                                                         C.byref(p)), "snapshot")
        return t.value, g.value, p.value

    def counters(self) -> gossip_counters:
        c = gossip_counters()
        _check(load_library().gossip_engine_get_counters(self._h, C.byref(c)), "counters")
        return c

    def reset_timing(self):
        _check(load_library().gossip_engine_reset_timing(self._h), "reset timing")

    def rehearsal(self, ranges: int) -> dict:
        """Option rehearse_rows = ranges: per row block, summed since reset_timing -- pull, pack
        and unpack time (ms) and message bytes, the number of ticks rehearsed, and the largest
        message of one tick (msg_bytes_max)."""
        pull, pack, unpack = (np.zeros(ranges) for _ in range(3))
        msg = np.zeros(ranges, np.uint64)
        ticks = C.c_uint64()
        _check(load_library().gossip_engine_get_rehearsal(self._h, ranges, _vp(pull), _vp(pack), _vp(unpack),
                                                          _vp(msg), C.byref(ticks)), "rehearsal")
        peak = np.zeros(ranges, np.uint64)
        _check(load_library().gossip_engine_get_rehearsal_peak(self._h, ranges, _vp(peak)), "rehearsal peak")
        return dict(pull_ms=pull, pack_ms=pack, unpack_ms=unpack, msg_bytes=msg, ticks=int(ticks.value),
                    msg_bytes_max=peak)

    def trace(self):
        lib = load_library()
        m = int(lib.gossip_engine_trace_size(self._h))
        node = np.empty(m, np.uint32)
        sid = np.empty(m, np.uint32)
        tick = np.empty(m, np.int64)
        hop = np.empty(m, np.uint32)
        via = np.empty(m, np.uint8)
        if m:
            _check(lib.gossip_engine_get_trace(self._h, _vp(node), _vp(sid), _vp(tick), _vp(hop),
                                               _vp(via)), "trace")
        return node, sid, tick, hop, via

    def close(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.gossip_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def format_event_log(topo: "Topology", ev: np.ndarray, trace, latency_ns: int, t_start_ns: int,
                     t_cut_ns: int, link_timing=None, with_time: bool = True):
    """The reference's NS_LOG_INFO gossip lines rendered from a first-contact trace
    (gossip.h, gossip_format_event_log).  trace = (node, share_id, tick, hop, via) as returned by
    Engine.trace(); ev = the run's generation events with real times.  Returns
    [(t_ns, line)] when with_time, else the plain text."""
    lib = load_library()
    ev = np.ascontiguousarray(ev, GEN_EVENT_DTYPE)
    node, sid, _tick, hop, via = (np.ascontiguousarray(x) for x in trace)
    node, sid, hop = (np.ascontiguousarray(x, np.uint32) for x in (node, sid, hop))
    via = np.ascontiguousarray(via, np.uint8)
    npb, hdr, dfr = link_timing or (0, 0, 0)
    args = [topo._h, ev.size, _vp(ev), node.size, _vp(node), _vp(sid), _vp(hop), _vp(via),
            int(latency_ns), int(t_start_ns), int(t_cut_ns), int(npb), int(hdr), int(dfr),
            1 if with_time else 0]
    ln = lib.gossip_format_event_log(*args, None, 0)
    _check(ln if ln < 0 else 0, "event log")
    buf = C.create_string_buffer(ln + 1)
    lib.gossip_format_event_log(*args, buf, ln + 1)
    text = buf.value.decode()
    if not with_time:
        return text
    out = []
    for line in text.splitlines():
        t, body = line.split("\t", 1)
        out.append((int(t), body))
    return out


def format_netanim(topo: "Topology", ev: np.ndarray, trace, latency_ns: int, t_cut_ns: int,
                   link_timing=None, packets: bool = True) -> str:
    """NetAnim XML of SetupNetAnim + EnablePacketMetadata (gossip.h, gossip_format_netanim): the
    node grid and links, and one <p> record per gossip Send derived from the first-contact trace
    (node, share_id, tick, hop, ...) of a run whose generation events are `ev`."""
    lib = load_library()
    ev = np.ascontiguousarray(ev, GEN_EVENT_DTYPE)
    node, sid, hop = (np.ascontiguousarray(trace[k], np.uint32) for k in (0, 1, 3))
    npb, hdr, dfr = link_timing or (0, 0, 0)
    args = [topo._h, ev.size, _vp(ev), node.size, _vp(node), _vp(sid), _vp(hop), int(latency_ns),
            int(t_cut_ns), int(npb), int(hdr), int(dfr), 1 if packets else 0]
    ln = lib.gossip_format_netanim(*args, None, 0)
    _check(ln if ln < 0 else 0, "netanim")
    buf = C.create_string_buffer(ln + 1)
    lib.gossip_format_netanim(*args, buf, ln + 1)
    return buf.value.decode()


def format_statistics(st: Stats) -> str:
    lib = load_library()
    n = st.gen.size
    args = [_vp(np.ascontiguousarray(x)) for x in
            (st.gen, st.recv, st.fwd, st.sent, st.processed, st.peers, st.sockets)]
    ln = lib.gossip_format_statistics(n, *args, None, 0)
    buf = C.create_string_buffer(ln + 1)
    lib.gossip_format_statistics(n, *args, buf, ln + 1)
    return buf.value.decode()


def format_periodic(t_seconds: float, n: int, total_gen: int, total_processed: int,
                    total_sockets: int) -> str:
    lib = load_library()
    ln = lib.gossip_format_periodic(t_seconds, n, total_gen, total_processed, total_sockets, None, 0)
    buf = C.create_string_buffer(ln + 1)
    lib.gossip_format_periodic(t_seconds, n, total_gen, total_processed, total_sockets, buf, ln + 1)
    return buf.value.decode()


class P2PGossipNetworkSimulation:
    """Mirror of the reference class (p2pnetwork.cc:15-286) driving the HIP engine.

    ``rd()`` is replaced by explicit seeds: ``topo_seed`` (p2pnetwork.cc:65) and
    ``node_seed`` (node i seeds ``node_seed + i``, p2pnode.cc:41).
    """

    def __init__(self, numNodes: int, topo_seed: int = 1, node_seed: int = 1000, device: int = 0,
                 topology_kind: int | None = None, threads: int = 8, flags: int = 0,
                 link_timing=None, shards: int = 1, options=None):
        if numNodes < 2:
            # p2pnetwork.cc:82 calls nodes.Get(1) for the fix-up of row 0: out of range.
            raise GossipError("numNodes < 2: the reference's topology fix-up aborts")
        self.numNodes = numNodes
        self.topo_seed = topo_seed
        self.node_seed = node_seed
        self.device = device
        self.kind = topology_kind
        self.threads = threads
        self.flags = flags
        self.link_timing = link_timing  # e.g. LINK_5MBPS (needs flags |= F_HOP_BATCH)
        self.shards = shards            # share shards run one after another on `device`
        self.options = dict(options or {})  # gossip_engine_set_option name -> value
        self.topology = None
        self.latency_ns = None
        self.engine = None
        self.periodic = []
        self.stats = None

    def CreateRandomTopology(self, connectionProbability: float = 0.3, latency: float = 5.0):
        kind = self.kind
        if kind is None:
            kind = TOPO_EXACT if self.numNodes <= 16384 else TOPO_SKIP
        self.topology = Topology.gnp(self.numNodes, connectionProbability, self.topo_seed, kind,
                                     self.threads)
        self.latency_ns = milliseconds_to_ns(latency)

    def _run_shard(self, ev, t_start, t_cut, snaps, rank, count):
        eng = Engine(self.numNodes, self.latency_ns, t_start, t_cut, device=self.device,
                     flags=self.flags, shard_rank=rank, shard_count=count)
        for k, v in self.options.items():
            eng.set_option(k, v)
        eng.set_topology(self.topology)
        if self.link_timing:
            eng.set_link_timing(*self.link_timing)
        for t in snaps:
            eng.add_snapshot(seconds_to_ns(t))
        eng.set_schedule(ev)
        eng.run()
        eng.sync()
        return eng

    def Start(self, simulationTime: float = 100.0, statsInterval: float = 10.0, events=None):
        """Run the simulation (p2pnetwork.cc:193-218).  The share instances run as `shards`
        engines one after another (counters add exactly); when an engine's live window does not
        fit the device (GOSSIP_ECAPACITY / GOSSIP_ENOMEM) the shard count doubles and the run
        restarts.  `events` (GEN_EVENT_DTYPE) replays a given schedule instead of the reference's
        (e.g. one dumped from an NS-3 run)."""
        if self.topology is None:
            raise GossipError("CreateRandomTopology first")
        t_start = seconds_to_ns(5.0)
        t_cut = seconds_to_ns(simulationTime - 0.1)
        ev = (make_schedule(self.numNodes, self.node_seed, t_start, t_cut, threads=self.threads)
              if events is None else np.ascontiguousarray(events, GEN_EVENT_DTYPE))
        times = []
        t = statsInterval
        while t < simulationTime:
            times.append(t)
            t += statsInterval
        count = max(1, int(self.shards))
        while True:
            try:
                parts = []
                for r in range(count):
                    eng = self._run_shard(ev, t_start, t_cut, times, r, count)
                    parts.append((eng.stats(), [eng.snapshot(k) for k in range(len(times))]))
                    if r + 1 < count:
                        eng.close()  # keep only the last engine (counters, trace) alive
                break
            except GossipError as e:
                if e.code not in (E_CAPACITY, E_NOMEM) or count >= 4096:
                    raise
                count *= 2
        self.shards_used = count
        self.engine = eng
        st = parts[0][0]
        if count > 1:  # counters add exactly over share shards
            st = Stats(*(sum(getattr(p[0], k).astype(np.uint64) for p in parts).astype(getattr(st, k).dtype)
                         if k not in ("peers", "sockets") else getattr(st, k)
                         for k in ("gen", "recv", "fwd", "sent", "processed", "peers", "sockets")))
        self.stats = st
        if t_cut < t_start:
            self.stats.peers[:] = 0
            self.stats.sockets[:] = 0
        total_sock = int(self.topology.degrees()[1].sum())
        self.periodic = []
        for k, ts in enumerate(times):
            tns = parts[0][1][k][0]
            g = sum(p[1][k][1] for p in parts)
            pr = sum(p[1][k][2] for p in parts)
            # sockets exist from makeconnections (t_start) until StopAllNodes (t_cut)
            live = t_start <= tns <= t_cut
            self.periodic.append((ts, g, pr, total_sock if live else 0))
        return self.stats

    def PrintPeriodicStats(self) -> str:
        return "".join(format_periodic(t, self.numNodes, g, p, s) for t, g, p, s in self.periodic)

    def PrintStatistics(self) -> str:
        return format_statistics(self.stats)
