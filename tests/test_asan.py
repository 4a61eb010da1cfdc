"""CPU sanitizer build: host.cpp / eventlog.cpp (the host C++ of libgossip.so) and both oracles
compiled with -fsanitize=address,undefined and driven by tests/asan/asan_driver.cpp -- topology
(exact stream == ORACLE A's links), schedule (== ORACLE A's generations), shard rule, report,
event log, NetAnim, ORACLE B == ORACLE A, and the strict dump loaders on malformed key and event
files (the reference's parser is UB on malformed input, p2pnode.cc:13-30; the ABI returns
GOSSIP_EINVAL).  Plus the gossip_sim CLI refusing malformed --links / --events dumps before it
touches a GPU."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG, ROOT

SIM = os.path.join(PKG, "lib", "gossip_sim")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ with libasan/libubsan")
def test_asan_ubsan_host_and_oracles(tmp_path):
    out = str(tmp_path / "asan")
    p = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "asan"), f"OUT={out}"],
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-4000:]
    assert "checks passed" in p.stdout
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr


@pytest.mark.parametrize("flag,text", [
    ("links", "0 1\n1 x\n"),
    ("links", "0 1\n2\n"),
    ("links", "0 12\n"),
    ("events", "5000000000 1\n"),
    ("events", "-5 1 2\n"),
    ("events", "5000000000 1 2 3\n"),
])
def test_cli_rejects_malformed_dumps(tmp_path, flag, text):
    f = tmp_path / "dump.txt"
    f.write_text(text)
    args = [SIM, "--numNodes=10", f"--{flag}={f}"]
    if flag == "events":
        good = tmp_path / "links.txt"
        good.write_text("0 1\n1 2\n")
        args.append(f"--links={good}")
    p = subprocess.run(args, capture_output=True, text=True, timeout=60)
    assert p.returncode != 0
    assert "line 1" in p.stderr or "line 2" in p.stderr, p.stderr
    assert "import failed" in p.stderr


def test_dump_loaders_round_trip(gossip, tmp_path):
    # --dumpLinks / --dumpEvents text read back through the strict ABI loaders
    import numpy as np

    topo = gossip.Topology.gnp(40, 0.2, 9, gossip.TOPO_EXACT)
    a, b = topo.links()
    f = tmp_path / "links.txt"
    f.write_text("".join(f"{x} {y}\n" for x, y in zip(a.tolist(), b.tolist())))
    back = gossip.Topology.load_links(40, str(f))
    a2, b2 = back.links()
    assert np.array_equal(a, a2) and np.array_equal(b, b2)
    ev = gossip.make_schedule(40, 3, 5_000_000_000, 9_900_000_000)
    g = tmp_path / "events.txt"
    g.write_text("".join(f"{t} {v} {i}\n" for t, v, i in zip(ev["ns"].tolist(), ev["node"].tolist(),
                                                             ev["share_id"].tolist())))
    assert np.array_equal(gossip.load_events(40, str(g)), ev)
    g.write_text("5000000000 1 2\n5000000000 x 2\n")
    with pytest.raises(gossip.GossipError, match="line 2"):
        gossip.load_events(40, str(g))
