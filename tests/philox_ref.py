"""Pure-numpy Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11; Random123) and the share
schedule rules of schedule_gpu.hip, as the independent checker of the GPU generator.  Test
infrastructure only."""
from fractions import Fraction

import numpy as np

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    """ctr: uint64 array (..., 4) of 32-bit words; key: (..., 2).  Returns (..., 4)."""
    c = [np.asarray(ctr[..., i], np.uint64) for i in range(4)]
    k0 = np.asarray(key[..., 0], np.uint64)
    k1 = np.asarray(key[..., 1], np.uint64)
    for _ in range(10):
        p0 = c[0] * np.uint64(M0)
        p1 = c[2] * np.uint64(M1)
        n0 = (p1 >> np.uint64(32)) ^ c[1] ^ k0
        n2 = (p0 >> np.uint64(32)) ^ c[3] ^ k1
        c = [n0 & np.uint64(MASK), p1 & np.uint64(MASK), n2 & np.uint64(MASK), p0 & np.uint64(MASK)]
        k0 = (k0 + np.uint64(W0)) & np.uint64(MASK)
        k1 = (k1 + np.uint64(W1)) & np.uint64(MASK)
    return np.stack(c, -1)


def seconds_to_ns(x: float) -> int:
    """ns-3 Seconds(): round-half-up of the exact product."""
    q = Fraction(x) * 1_000_000_000
    return int(q + Fraction(1, 2)) if q >= 0 else -int(-q + Fraction(1, 2))


KEY1 = 0x53484152
C2, C3 = 0x676F7373, 0x69702D73


def node_events(v, seed, t_start, t_end):
    """(ns, id) of node v's counted generations under schedule_gpu.hip's rules."""
    out = []
    t, g, blk, buf = 0, 0, 0, []
    def draw():
        nonlocal blk, buf
        if not buf:
            ctr = np.array([[v, blk, C2, C3]], np.uint64)
            key = np.array([[seed, KEY1]], np.uint64)
            buf = [int(x) for x in philox4x32_10(ctr, key)[0]]
            blk += 1
        return buf.pop(0)
    while True:
        x0, x1 = draw(), draw()
        u = (x0 + x1 * 2.0 ** 32) * 2.0 ** -64
        if u >= 1.0:
            u = float.fromhex("0x1.fffffffffffffp-1")
        t += seconds_to_ns(2.0 + u * 3.0)
        if t >= t_end:
            return out
        if t < t_start:
            continue
        out.append((t, (v * 1_000_000 + g * 1000 + t % 1000) & MASK))
        g += 1
