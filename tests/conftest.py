import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "p2p-gossip-simulation-ns3_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


def _stale(target, srcs):
    # missing, or a source edited after the build (60 s of slack: a copied tree whose files all
    # got one extraction time is not "stale")
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(f) > t + 60 for f in srcs if os.path.exists(f))


def _ensure_built():
    # a libgossip.so older than its sources is rebuilt, never tested; a fresh tree is left alone
    csrc = os.path.join(PKG, "csrc")
    srcs = [os.path.join(csrc, f) for f in os.listdir(csrc)] + [os.path.join(ROOT, "include", "gossip.h")]
    odir = os.path.join(ROOT, "oracle")
    osrcs = [os.path.join(odir, f) for f in ("oracle.cpp", "oracle_b.cpp", "oracle.h", "Makefile")]
    for d, target, ss in ((odir, os.path.join(odir, "liboracle.so"), osrcs),
                          (csrc, os.path.join(PKG, "lib", "libgossip.so"), srcs)):
        if _stale(target, ss):
            print(f"conftest: {target} missing or older than its sources, rebuilding", file=sys.stderr)
            subprocess.run(["make", "-s", "-C", d], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def gossip():
    import gossip as g
    g.load_library()
    return g


class _MemoOracle:
    """The oracle module with run_replay memoised on its arguments' bytes: parametrized GPU tests
    that vary only engine options over one workload run ORACLE A once (its single-threaded replay
    is most of their time on the GPU box).  Results are shared, never modified by the tests."""

    def __init__(self, mod):
        self._mod = mod
        self._memo = {}

    def __getattr__(self, name):
        return getattr(self._mod, name)

    @staticmethod
    def _key(args, kw):
        import hashlib

        import numpy as np
        h = hashlib.blake2b(digest_size=20)
        for x in list(args) + sorted(kw.items()):
            if isinstance(x, np.ndarray):
                h.update(repr((x.dtype.str, x.shape)).encode())
                h.update(np.ascontiguousarray(x).tobytes())
            else:
                h.update(repr(x).encode())
            h.update(b"|")
        return h.digest()

    def run_replay(self, *args, **kw):
        k = self._key(args, kw)
        if k not in self._memo:
            if len(self._memo) >= 48:
                self._memo.pop(next(iter(self._memo)))
            self._memo[k] = self._mod.run_replay(*args, **kw)
        return self._memo[k]


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.load()
    return _MemoOracle(o)
