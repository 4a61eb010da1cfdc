"""ctypes binding of ORACLE A (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker / the timed CPU baseline, never as the product.
Parity status: unpinned against NS-3 (see oracle.h and DESIGN.md "Oracle").
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
INT64_MAX = (1 << 63) - 1

_lib = None


class oracle_params(C.Structure):
    _fields_ = [
        ("num_nodes", C.c_uint32), ("connection_prob", C.c_double), ("sim_time_s", C.c_double),
        ("latency_ms", C.c_double), ("topo_seed", C.c_uint32), ("node_seed", C.c_uint32),
        ("id_mask", C.c_uint32), ("register_delay_ns", C.c_int64), ("est_delay_ns", C.c_int64),
    ]


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: build with `make -C oracle`")
        lib = C.CDLL(LIB_PATH)
        P = C.c_void_p
        lib.oracle_create_reference.argtypes = [C.POINTER(oracle_params), C.POINTER(P)]
        lib.oracle_create_replay.argtypes = [C.c_uint32, C.c_int64, C.c_int64, C.c_int64,
                                             C.c_uint64, P, P, C.c_uint64, P, P, P, C.POINTER(P)]
        lib.oracle_enable_trace.argtypes = [P]
        lib.oracle_enable_log.argtypes = [P]
        lib.oracle_get_log.argtypes = [P, C.c_char_p, C.c_uint64]
        lib.oracle_get_log.restype = C.c_int64
        lib.oracle_set_handshake.argtypes = [P, C.c_int64, C.c_int64]
        lib.oracle_set_link_timing.argtypes = [P, C.c_int64, C.c_uint32, C.c_int64]
        lib.oracle_run.argtypes = [P]
        lib.oracle_get_stats.argtypes = [P] + [P] * 7
        lib.oracle_get_counters.argtypes = [P, P, P, P]
        lib.oracle_get_links.argtypes = [P, P, P]
        lib.oracle_get_links.restype = C.c_uint64
        lib.oracle_get_gen_events.argtypes = [P, P, P, P]
        lib.oracle_get_gen_events.restype = C.c_uint64
        lib.oracle_get_periodic.argtypes = [P, P, P, P, P]
        lib.oracle_get_periodic.restype = C.c_uint64
        lib.oracle_get_trace.argtypes = [P, P, P, P, P, P]
        lib.oracle_get_trace.restype = C.c_uint64
        lib.oracle_seconds_to_ns.argtypes = [C.c_double]
        lib.oracle_seconds_to_ns.restype = C.c_int64
        lib.oracle_milliseconds_to_ns.argtypes = [C.c_double]
        lib.oracle_milliseconds_to_ns.restype = C.c_int64
        lib.oracle_last_error.restype = C.c_char_p
        lib.oracle_destroy.argtypes = [P]
        lib.oracle_b_run.argtypes = [C.c_uint32, C.c_int64, C.c_int64, C.c_uint64, P, P, C.c_uint64,
                                     P, P, P, C.c_int] + [P] * 8
        lib.oracle_b_last_error.restype = C.c_char_p
        lib.oracle_b_last_wall_s.restype = C.c_double
        _lib = lib
    return _lib


def _vp(a):
    return C.c_void_p(a.ctypes.data) if a is not None and a.size else None


@dataclass
class OracleResult:
    gen: np.ndarray
    recv: np.ndarray
    fwd: np.ndarray
    sent: np.ndarray
    processed: np.ndarray
    peers: np.ndarray
    sockets: np.ndarray
    edge_events: int
    events: int
    wall_s: float
    links: tuple
    gen_events: tuple
    periodic: list
    trace: tuple | None
    log: list | None = None  # [(t_ns, NS_LOG_INFO line)] in event order (log=True)


class OracleSim:
    def __init__(self, handle, n):
        self._h = C.c_void_p(handle)
        self.n = n

    @classmethod
    def reference(cls, num_nodes, connection_prob=0.3, sim_time_s=60.0, latency_ms=5.0,
                  topo_seed=1, node_seed=1000, id_mask=0, register_delay_ns=0, est_delay_ns=0):
        lib = load()
        p = oracle_params(num_nodes, connection_prob, sim_time_s, latency_ms, topo_seed, node_seed,
                          id_mask, register_delay_ns, est_delay_ns)
        h = C.c_void_p()
        if lib.oracle_create_reference(C.byref(p), C.byref(h)) != 0:
            raise RuntimeError(lib.oracle_last_error().decode())
        return cls(h.value, num_nodes)

    @classmethod
    def replay(cls, num_nodes, latency_ns, t_start_ns, t_cut_ns, link_a, link_b, ev_ns, ev_node,
               ev_id):
        lib = load()
        a = np.ascontiguousarray(link_a, np.uint32)
        b = np.ascontiguousarray(link_b, np.uint32)
        ns = np.ascontiguousarray(ev_ns, np.int64)
        nd = np.ascontiguousarray(ev_node, np.uint32)
        ids = np.ascontiguousarray(ev_id, np.uint32)
        h = C.c_void_p()
        rc = lib.oracle_create_replay(num_nodes, latency_ns, t_start_ns, t_cut_ns, a.size, _vp(a),
                                      _vp(b), ns.size, _vp(ns), _vp(nd), _vp(ids), C.byref(h))
        if rc != 0:
            raise RuntimeError(lib.oracle_last_error().decode())
        return cls(h.value, num_nodes)

    def enable_trace(self):
        load().oracle_enable_trace(self._h)

    def enable_log(self):
        load().oracle_enable_log(self._h)

    def get_log(self):
        lib = load()
        k = lib.oracle_get_log(self._h, None, 0)
        b = C.create_string_buffer(k + 1)
        lib.oracle_get_log(self._h, b, k + 1)
        out = []
        for ln in b.value.decode().splitlines():
            t, txt = ln.split("\t", 1)
            out.append((int(t), txt))
        return out

    def run(self, want_trace=False) -> OracleResult:
        lib = load()
        lib.oracle_run(self._h)
        n = self.n
        u = [np.empty(n, np.uint32) for _ in range(6)]
        sent = np.empty(n, np.uint64)
        lib.oracle_get_stats(self._h, _vp(u[0]), _vp(u[1]), _vp(u[2]), _vp(sent), _vp(u[3]),
                             _vp(u[4]), _vp(u[5]))
        ee, evn, wall = C.c_uint64(), C.c_uint64(), C.c_double()
        lib.oracle_get_counters(self._h, C.byref(ee), C.byref(evn), C.byref(wall))
        m = lib.oracle_get_links(self._h, None, None)
        la, lb = np.empty(m, np.uint32), np.empty(m, np.uint32)
        lib.oracle_get_links(self._h, _vp(la), _vp(lb))
        m = lib.oracle_get_gen_events(self._h, None, None, None)
        gns, gnode, gid = np.empty(m, np.int64), np.empty(m, np.uint32), np.empty(m, np.uint32)
        lib.oracle_get_gen_events(self._h, _vp(gns), _vp(gnode), _vp(gid))
        m = lib.oracle_get_periodic(self._h, None, None, None, None)
        pt, pg, pp, ps = (np.empty(m, np.int64), np.empty(m, np.uint32), np.empty(m, np.uint32),
                          np.empty(m, np.uint32))
        lib.oracle_get_periodic(self._h, _vp(pt), _vp(pg), _vp(pp), _vp(ps))
        periodic = [(int(pt[k]), int(pg[k]), int(pp[k]), int(ps[k])) for k in range(m)]
        trace = None
        if want_trace:
            m = lib.oracle_get_trace(self._h, None, None, None, None, None)
            tn, ti, tt, th, tv = (np.empty(m, np.uint32), np.empty(m, np.uint32),
                                  np.empty(m, np.int64), np.empty(m, np.uint32),
                                  np.empty(m, np.uint8))
            lib.oracle_get_trace(self._h, _vp(tn), _vp(ti), _vp(tt), _vp(th), _vp(tv))
            trace = (tn, ti, tt, th, tv)
        return OracleResult(u[0], u[1], u[2], sent, u[3], u[4], u[5], ee.value, evn.value,
                            wall.value, (la, lb), (gns, gnode, gid), periodic, trace)

    def close(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.oracle_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


# NS-3 5 Mbps point-to-point links (p2pnetwork.cc:113): ns per byte, PPP+IPv4+TCP(ts option)
# header bytes, TcpSocketBase's one-TimeStep send deferral
LINK_5MBPS = (1600, 54, 1)


def _set_link_timing(s, link_timing):
    if link_timing:
        if load().oracle_set_link_timing(s._h, *(int(x) for x in link_timing)) != 0:
            raise RuntimeError(load().oracle_last_error().decode())


def _run(s, trace, log):
    if trace:
        s.enable_trace()
    if log:
        s.enable_log()
    try:
        r = s.run(want_trace=trace)
        if log:
            r.log = s.get_log()
        return r
    finally:
        s.close()


def run_reference(**kw) -> OracleResult:
    trace = kw.pop("trace", False)
    log = kw.pop("log", False)
    link_timing = kw.pop("link_timing", None)
    s = OracleSim.reference(**kw)
    _set_link_timing(s, link_timing)
    return _run(s, trace, log)


def run_replay(*args, trace=False, handshake=None, link_timing=None, log=False) -> OracleResult:
    """handshake = (est_delay_ns, register_delay_ns): the NS-3 handshake-window model.
    link_timing = (ns_per_byte, header_bytes, send_defer_ns), e.g. LINK_5MBPS."""
    s = OracleSim.replay(*args)
    _set_link_timing(s, link_timing)
    if handshake:
        if load().oracle_set_handshake(s._h, int(handshake[0]), int(handshake[1])) != 0:
            raise RuntimeError(load().oracle_last_error().decode())
    return _run(s, trace, log)


def run_oracle_b(num_nodes, latency_ns, t_cut_ns, link_a, link_b, ev_ns, ev_node, ev_id,
                 threads=8) -> OracleResult:
    """ORACLE B (oracle_b.cpp): bit-sliced level-synchronous restatement for schedules with
    distinct share ids; same inputs as run_replay (t_start is implicit: every edge is up before
    the first counted generation).  Stats only (no trace / periodic)."""
    lib = load()
    n = int(num_nodes)
    a = np.ascontiguousarray(link_a, np.uint32)
    b = np.ascontiguousarray(link_b, np.uint32)
    ns = np.ascontiguousarray(ev_ns, np.int64)
    nd = np.ascontiguousarray(ev_node, np.uint32)
    ids = np.ascontiguousarray(ev_id, np.uint32)
    u = [np.empty(n, np.uint32) for _ in range(6)]
    sent = np.empty(n, np.uint64)
    ee = C.c_uint64()
    rc = lib.oracle_b_run(n, int(latency_ns), int(t_cut_ns), a.size, _vp(a), _vp(b), ns.size,
                          _vp(ns), _vp(nd), _vp(ids), int(threads), _vp(u[0]), _vp(u[1]),
                          _vp(u[2]), _vp(sent), _vp(u[3]), _vp(u[4]), _vp(u[5]), C.byref(ee))
    if rc != 0:
        raise RuntimeError(lib.oracle_b_last_error().decode())
    # wall_s: the bit-sliced propagation only (CSR construction excluded)
    return OracleResult(u[0], u[1], u[2], sent, u[3], u[4], u[5], ee.value, int(ns.size),
                        float(lib.oracle_b_last_wall_s()), (a, b), (ns, nd, ids), [], None)


def seconds_to_ns(s):
    return int(load().oracle_seconds_to_ns(float(s)))


def milliseconds_to_ns(ms):
    return int(load().oracle_milliseconds_to_ns(float(ms)))
