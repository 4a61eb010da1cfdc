"""The gossip_sim CLI (replacement of the reference's main(), p2pnetwork.cc:289-313): NetAnim
export (SetupNetAnim + EnablePacketMetadata, p2pnetwork.cc:153-190) from ORACLE A's trace here and
from the GPU run on the box, and on the GPU the report text and the first-contact trace dump
against ORACLE A."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG

SIM = os.path.join(PKG, "lib", "gossip_sim")


def _check_topology_xml(gossip, xml):
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


P_RE = re.compile(r'<p fId="(\d+)" fbTx="([\d.]+)" lbTx="([\d.]+)" meta-info="SHARE:(\d+):(\d+):([^"]+)" '
                  r'tId="(\d+)" fbRx="([\d.]+)" lbRx="([\d.]+)" />')


@pytest.mark.parametrize("link", [False, True])
def test_netanim_packets_from_oracle_trace(gossip, oracle, link):
    # The packet records (EnablePacketMetadata, p2pnetwork.cc:187) rendered from ORACLE A's
    # first-contact trace: one <p> per Send, so per node they must add up to its "Total shares
    # sent" (p2pnode.cc:140), with the link model's times.
    n, p, L = 30, 0.2, 5_000_000
    topo = gossip.Topology.gnp(n, p, 5, gossip.TOPO_EXACT)
    t0, t_cut = gossip.seconds_to_ns(5.0), gossip.seconds_to_ns(11.9)
    ev = gossip.make_schedule(n, 6, t0, t_cut)
    a, b = topo.links()
    lt = gossip.LINK_5MBPS if link else None
    r = oracle.run_replay(n, L, t0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"], trace=True,
                          link_timing=lt)
    xml = gossip.format_netanim(topo, ev, r.trace, L, t_cut, link_timing=lt)
    _check_topology_xml(gossip, xml)
    recs = P_RE.findall(xml)
    assert len(recs) == int(r.sent.sum()) > 0
    per = np.bincount([int(x[0]) for x in recs], minlength=n)
    assert np.array_equal(per, r.sent.astype(np.int64))
    peers = r.peers
    for f, fb, lb, o, sid, ts, to, fr, lr in recs[:200]:
        fb, lb, fr, lr = float(fb), float(lb), float(fr), float(lr)
        msg = f"SHARE:{o}:{sid}:{ts}"
        assert abs((fr - fb) - L / 1e9) < 1e-9 and abs((lr - lb) - L / 1e9) < 1e-9
        wire = (len(msg) + 54) * 1600 / 1e9 if link else 0.0
        assert abs((lb - fb) - wire) < 1e-9
        assert peers[int(f)] > 0
    assert xml.rstrip().endswith("</anim>")
    assert gossip.format_netanim(topo, ev, r.trace, L, t_cut, packets=False).count("<p ") == 0


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


@pytest.mark.gpu
def test_cli_netanim_with_packets(gossip, oracle, tmp_path):
    out = tmp_path / "anim.xml"
    p = subprocess.run([SIM, "--numNodes=30", "--connectionProb=0.2", "--seed=5", "--nodeSeed=7",
                        "--simTime=12", f"--netanim={out}"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert f"NetAnim configured to save in {out}" in p.stdout
    xml = out.read_text()
    _check_topology_xml(gossip, xml)
    r = oracle.run_reference(num_nodes=30, connection_prob=0.2, sim_time_s=12.0, topo_seed=5, node_seed=7)
    recs = P_RE.findall(xml)
    assert len(recs) == int(r.sent.sum()) > 0


@pytest.mark.gpu
def test_cli_rows_rank_failure_does_not_hang():
    # --layout=rows, 2 ranks: on a 1-GPU box rank 1 cannot create its engine.  Rank 0 must not
    # wait forever in ncclCommInitRank for it (the ranks meet before RCCL init and fail together).
    p = subprocess.run([SIM, "--numNodes=3000", "--connectionProb=0.01", "--simTime=6", "--gpus=2",
                        "--layout=rows", "--quiet"], capture_output=True, text=True, timeout=180)
    if p.returncode == 0:  # a box with two visible GPUs ran the partition
        assert "row ranks (RCCL exchange)" in p.stdout
        return
    assert "engine create" in p.stderr, p.stderr
