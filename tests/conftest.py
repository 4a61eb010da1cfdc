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


def _ensure_built():
    libs = [os.path.join(ROOT, "oracle", "liboracle.so"), os.path.join(PKG, "lib", "libgossip.so")]
    if all(os.path.exists(p) for p in libs):
        return
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def gossip():
    import gossip as g
    g.load_library()
    return g


@pytest.fixture(scope="session")
def oracle():
    import oracle as o
    o.load()
    return o
