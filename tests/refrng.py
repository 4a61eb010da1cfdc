"""Pure-Python restatement of the libstdc++ random pieces the reference uses.

Test helper only.  It pins the C++ oracle and the product host code to the published
algorithms independently of the C++ standard library they are compiled against:

* std::mt19937 (C++11 [rand.eng.mers], seed(s) per [rand.eng.mers]/8); KAT: the 10000th
  output of a default-constructed engine is 4123659995 ([rand.predef]/3).
* std::generate_canonical<double, 53> as libstdc++ 11 implements it
  (/usr/include/c++/11/bits/random.tcc:3348-3381): k = 2 draws, (x0 + x1*2^32) / 2^64,
  clamped below 1.
* std::uniform_real_distribution<double>(a, b): a + u*(b-a) (bits/random.h:1866-1871 via
  _Adaptor, bits/random.h:164-194).
* ns-3 Seconds(double): round-half-up of the exact product value*1e9 (int64x64 path).
"""
from fractions import Fraction


class MT19937:
    N, M = 624, 397

    def __init__(self, seed=5489):
        self.seed(seed)

    def seed(self, s):
        s &= 0xFFFFFFFF
        mt = [0] * self.N
        mt[0] = s
        for i in range(1, self.N):
            mt[i] = (1812433253 * (mt[i - 1] ^ (mt[i - 1] >> 30)) + i) & 0xFFFFFFFF
        self.mt = mt
        self.idx = self.N

    def _twist(self):
        mt = self.mt
        for i in range(self.N):
            y = (mt[i] & 0x80000000) | (mt[(i + 1) % self.N] & 0x7FFFFFFF)
            v = mt[(i + self.M) % self.N] ^ (y >> 1)
            if y & 1:
                v ^= 0x9908B0DF
            mt[i] = v
        self.idx = 0

    def __call__(self):
        if self.idx >= self.N:
            self._twist()
        y = self.mt[self.idx]
        self.idx += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF


def generate_canonical(g) -> float:
    x0 = float(g())
    x1 = float(g())
    s = x0 + x1 * 4294967296.0  # double arithmetic, as libstdc++ sums in _RealType
    r = s / 18446744073709551616.0
    if r >= 1.0:
        import math
        r = math.nextafter(1.0, 0.0)
    return r


def uniform_real(g, a, b) -> float:
    return generate_canonical(g) * (b - a) + a


def seconds_to_ns(x: float) -> int:
    """round-half-up of the exact rational x * 1e9 (x a double)."""
    q = Fraction(x) * 1_000_000_000
    neg = q < 0
    q = abs(q)
    r = int(q + Fraction(1, 2))  # floor(q + 1/2)
    return -r if neg else r


def node_schedule(node, node_seed, t_start_ns, t_cut_ns):
    """Counted generations of one node: [(ns, shareId)] (p2pnode.cc:33-43, 97-125, 201-209)."""
    g = MT19937((node_seed + node) & 0xFFFFFFFF)
    t = 0
    out = []
    gcount = 0
    while True:
        t += seconds_to_ns(uniform_real(g, 2.0, 5.0))
        if t >= t_cut_ns:
            return out
        if t < t_start_ns:
            continue
        sid = (node * 1_000_000 + gcount * 1000 + t % 1000) & 0xFFFFFFFF
        out.append((t, sid))
        gcount += 1


def topology_links(n, p, seed):
    """CreateRandomTopology key list (p2pnetwork.cc:62-96)."""
    g = MT19937(seed)
    links = []
    for i in range(n):
        connected = False
        for j in range(i + 1, n):
            if generate_canonical(g) < p:
                connected = True
                links.append((i, j))
        if not connected:
            links.append((0, 1) if i == 0 else (i, i - 1))
    return sorted(links)
