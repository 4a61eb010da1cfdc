"""The C-ABI library loads and exports every entry point include/gossip.h declares; the
engine refuses to run without a HIP device (no CPU fallback)."""
import ctypes
import os
import re

import pytest

from conftest import PKG, ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "gossip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gossip_[a-z0-9_]+)\s*\(", src)))


def test_every_declared_symbol_is_exported(gossip):
    lib = ctypes.CDLL(os.path.join(PKG, "lib", "libgossip.so"))
    names = _declared()
    assert len(names) >= 35
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # and the Python binding knows all of them
    assert set(names) <= set(gossip.EXPORTED_SYMBOLS)


def test_version_and_errors(gossip):
    lib = gossip.load_library()
    assert lib.gossip_version().decode().startswith("gossip-mi355x")
    with pytest.raises(gossip.GossipError, match="numNodes < 2"):
        gossip.Topology.gnp(1, 0.3, 1)


def _has_device():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_device(), reason="a GPU is present: the no-device path is not reachable")
def test_engine_refuses_without_device(gossip):
    with pytest.raises(gossip.GossipError, match="no HIP device|HIP"):
        gossip.Engine(10, 5_000_000, 5_000_000_000, 59_900_000_000)


def test_engine_rejects_bad_latency(gossip):
    # generation intervals are U(2,5) s (p2pnode.cc:99): one generation per node per tick
    # needs latency < 2 s; the check runs before any device query.
    with pytest.raises(gossip.GossipError, match="latency"):
        gossip.Engine(10, 2_000_000_000, 5_000_000_000, 59_900_000_000)
