"""GPU Philox share-generation (schedule_gpu.hip, gossip_schedule_create_philox) against an
independent numpy restatement (tests/philox_ref.py), whose Philox4x32-10 is pinned by the
Random123 known-answer vectors."""
import numpy as np
import pytest

import philox_ref as P

T0 = 5_000_000_000

KAT = [  # Random123 kat_vectors: philox4x32 10 (ctr, key) -> out
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_reference_philox_kat(ctr, key, want):
    got = P.philox4x32_10(np.array([ctr], np.uint64), np.array([key], np.uint64))[0]
    assert [int(x) for x in got] == list(want)


def test_reference_seconds_rounding():
    assert P.seconds_to_ns(2.0) == 2_000_000_000
    assert P.seconds_to_ns(2.0 ** -10) == 976563  # 976562.5 rounds half up (ns-3 int64x64)


@pytest.mark.gpu
def test_gpu_schedule_matches_reference(gossip):
    n, seed = 600, 77
    t_cut = gossip.seconds_to_ns(59.9)
    ev = gossip.make_schedule_philox(n, seed, T0, t_cut)
    want = sorted((t, v, i) for v in range(n) for t, i in P.node_events(v, seed, T0, t_cut))
    got = list(zip(ev["ns"].tolist(), ev["node"].tolist(), ev["share_id"].tolist()))
    assert got == want


@pytest.mark.gpu
def test_gpu_schedule_window_and_rate(gossip):
    n = 1_000_000
    t_end = T0 + gossip.seconds_to_ns(2.0)
    ev = gossip.make_schedule_philox(n, 5, T0, gossip.seconds_to_ns(59.9), t_gen_end_ns=t_end)
    assert ev["ns"].min() >= T0 and ev["ns"].max() < t_end
    assert np.all(np.diff(ev["ns"]) >= 0)
    same = np.diff(ev["ns"]) == 0
    assert np.all(np.diff(ev["node"].astype(np.int64))[same] > 0)  # (ns, node) order
    # the same renewal process as the reference's mt19937 schedule (started at t = 0, not yet
    # stationary at 5-7 s): the two event counts agree to sampling noise (~0.15 %)
    ref = gossip.make_schedule(n, 5, T0, gossip.seconds_to_ns(59.9), t_gen_end_ns=t_end, threads=16)
    assert abs(len(ev) / len(ref) - 1.0) < 0.01
    # a node's events are >= 2 s apart: at most one per node in a 2 s window
    assert len(np.unique(ev["node"])) == len(ev)


@pytest.mark.gpu
def test_cli_philox_schedule(gossip, oracle, tmp_path):
    # gossip_sim --schedule=philox: the dumped schedule is the library's, the report the oracle's
    import os
    import subprocess

    from conftest import PKG

    evf = tmp_path / "ev.txt"
    sim = os.path.join(PKG, "lib", "gossip_sim")
    p = subprocess.run([sim, "--numNodes=300", "--connectionProb=0.03", "--simTime=14", "--seed=4",
                        "--nodeSeed=9", "--schedule=philox", f"--dumpEvents={evf}"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    got = np.loadtxt(evf, dtype=np.int64).reshape(-1, 3)
    t_cut = gossip.seconds_to_ns(13.9)
    ev = gossip.make_schedule_philox(300, 9, T0, t_cut)
    assert np.array_equal(got[:, 0], ev["ns"]) and np.array_equal(got[:, 1], ev["node"])
    assert np.array_equal(got[:, 2], ev["share_id"])
    topo = gossip.Topology.gnp(300, 0.03, 4, gossip.TOPO_EXACT)
    a, b = topo.links()
    r = oracle.run_replay(300, 5_000_000, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"])
    want = gossip.format_statistics(gossip.Stats(r.gen, r.recv, r.fwd, r.sent, r.processed, r.peers,
                                                 r.sockets))
    assert want in p.stdout


@pytest.mark.gpu
def test_engine_runs_a_philox_schedule_like_the_oracle(gossip, oracle):
    n = 500
    topo = gossip.Topology.gnp(n, 0.02, 12, gossip.TOPO_EXACT)
    t_cut = gossip.seconds_to_ns(15.0)
    ev = gossip.make_schedule_philox(n, 13, T0, t_cut)
    eng = gossip.Engine(n, 5_000_000, T0, t_cut)
    eng.set_topology(topo)
    eng.set_schedule(ev)
    eng.run()
    st = eng.stats()
    a, b = topo.links()
    r = oracle.run_replay(n, 5_000_000, T0, t_cut, a, b, ev["ns"], ev["node"], ev["share_id"])
    for k in ("gen", "recv", "fwd", "sent", "processed"):
        assert np.array_equal(getattr(st, k), getattr(r, k)), k
    eng.close()
