"""The gossip_sim CLI (replacement of the reference's main(), p2pnetwork.cc:289-313): NetAnim
export (SetupNetAnim, p2pnetwork.cc:153-190), and on the GPU the report text and the
first-contact trace dump against ORACLE A."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG

SIM = os.path.join(PKG, "lib", "gossip_sim")


def test_netanim_export(gossip, tmp_path):
    out = tmp_path / "anim.xml"
    subprocess.run([SIM, "--numNodes=30", "--connectionProb=0.2", "--seed=5", f"--netanim={out}"],
                   capture_output=True, timeout=60)  # the engine itself needs a GPU; the XML does not
    xml = out.read_text()
    nodes = re.findall(r'<node id="(\d+)" sysId="0" locX="(\d+)" locY="(\d+)" />', xml)
    assert len(nodes) == 30
    grid = 6  # ceil(sqrt(30)), p2pnetwork.cc:160
    for i, x, y in nodes:
        assert (int(x), int(y)) == (100 * (int(i) % grid), 100 * (int(i) // grid))
    # SetupNetAnim runs in Start() before makeconnections: every node has 0 peers -> blue
    assert len(re.findall(r'r="0" g="0" b="255"', xml)) == 30
    a, b = gossip.Topology.gnp(30, 0.2, 5, gossip.TOPO_EXACT).links()
    links = re.findall(r'<link fromId="(\d+)" toId="(\d+)"', xml)
    assert [(int(x), int(y)) for x, y in links] == list(zip(a.tolist(), b.tolist()))


@pytest.mark.gpu
def test_cli_report_and_trace_match_oracle(gossip, oracle, tmp_path):
    tr = tmp_path / "trace.txt"
    p = subprocess.run([SIM, "--numNodes=10", "--seed=3", "--nodeSeed=3000", f"--dumpTrace={tr}"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    r = oracle.run_reference(num_nodes=10, connection_prob=0.3, sim_time_s=60.0, topo_seed=3,
                             node_seed=3000, trace=True)
    want = gossip.format_statistics(gossip.Stats(r.gen, r.recv, r.fwd, r.sent, r.processed, r.peers,
                                                 r.sockets))
    assert want in p.stdout
    d = np.loadtxt(tr, dtype=np.int64).reshape(-1, 5)
    tn, ti, tt, th, tv = r.trace
    ek, ok = np.lexsort((d[:, 1], d[:, 0])), np.lexsort((ti, tn))
    assert np.array_equal(d[ek, 0], tn[ok]) and np.array_equal(d[ek, 1], ti[ok])
    assert np.array_equal(d[ek, 2], tt[ok] // 5_000_000) and np.array_equal(d[ek, 3], th[ok])
    assert np.array_equal(d[ek, 4], tv[ok])
