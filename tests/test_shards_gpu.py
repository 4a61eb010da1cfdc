"""Share shards as the drop-in main() runs them, and the capacity fallback.

gossip_sim --gpus/--shards (one host thread per device, shards summed on the host) and
P2PGossipNetworkSimulation(shards=...) must print exactly the single-engine report, and when a
shard's live window does not fit its memory budget (engine option mem_limit) both must split the
shares into more shards on their own instead of failing (GOSSIP_ECAPACITY / GOSSIP_ENOMEM).
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG

pytestmark = pytest.mark.gpu

SIM = os.path.join(PKG, "lib", "gossip_sim")
STATS = ("gen", "recv", "fwd", "sent", "processed", "peers", "sockets")


def _sim(*args):
    p = subprocess.run([SIM, *args], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    return p


def _report(stdout):
    # everything but the engine-layout line
    return "\n".join(ln for ln in stdout.splitlines() if not ln.startswith("engines:"))


def test_cli_shards_print_the_single_engine_report(gossip, oracle):
    base = ["--numNodes=300", "--connectionProb=0.02", "--simTime=12", "--seed=7", "--nodeSeed=70"]
    one = _sim(*base)
    r = oracle.run_reference(num_nodes=300, connection_prob=0.02, sim_time_s=12.0, topo_seed=7, node_seed=70)
    want = gossip.format_statistics(gossip.Stats(r.gen, r.recv, r.fwd, r.sent, r.processed, r.peers,
                                                 r.sockets))
    assert want in one.stdout
    for shards in (2, 5):
        many = _sim(*base, f"--shards={shards}")
        assert f"engines: {shards} share shards" in many.stdout
        assert _report(many.stdout) == _report(one.stdout)


N_BURST = 20000
T0 = 5_000_000_000


def _burst(gossip):
    """4,096 distinct shares born in one tick of a 20,000-node sparse graph: one engine's window
    must hold all of them, each of 2 shards about half (tools/diag/shard_fallback.py)."""
    rng = np.random.Generator(np.random.Philox(11))
    nodes = rng.choice(N_BURST, size=4096, replace=False)
    return gossip.events_from_arrays(T0 + 1000 + np.arange(4096, dtype=np.int64), nodes,
                                     np.arange(1, 4097, dtype=np.uint32))


def _budget(gossip, ev):
    """A device-memory budget that one engine cannot meet for the burst and each of 2 shards can,
    from the engines' own reported need (gossip_counters.device_bytes) -- not a constant, so the
    test follows any change of the engine's layout.  Under a budget an engine allocates its window
    estimate without the headroom an unbudgeted one adds (engine.hip) and fails with
    GOSSIP_ECAPACITY when that does not fit, so the budget lies between what 2 shards and what 1
    engine allocate under a budget."""
    topo = gossip.Topology.gnp(N_BURST, 16.0 / (N_BURST - 1), 8, gossip.TOPO_SKIP)
    t_cut = gossip.seconds_to_ns(5.2)

    def need(shards, r):
        eng = gossip.Engine(N_BURST, 5_000_000, T0, t_cut, shard_rank=r, shard_count=shards)
        eng.set_option("mem_limit", 1 << 30)  # (a budget: no headroom)
        eng.set_topology(topo)
        eng.set_schedule(ev)
        eng.run()
        eng.sync()
        c = eng.counters()
        eng.close()
        return c.device_bytes

    one = need(1, 0)
    two = max(need(2, r) for r in range(2))
    mib = (one + two) // 2 >> 20  # (the CLI takes whole MB)
    assert two < mib << 20 < one, (one, two, mib)
    return mib


def test_cli_falls_back_to_more_shards(gossip, tmp_path):
    ev = _burst(gossip)
    evf = tmp_path / "ev.txt"
    np.savetxt(evf, np.stack([ev["ns"], ev["node"], ev["share_id"]], 1), fmt="%d")
    base = [f"--numNodes={N_BURST}", f"--connectionProb={16.0 / (N_BURST - 1)}", "--simTime=5.3",
            "--seed=8", f"--events={evf}", "--quiet"]
    one = _sim(*base)
    lim = _sim(*base, f"--memLimitMB={_budget(gossip, ev)}")
    assert "retrying with 2" in lim.stderr
    assert "engines: 2 share shards" in lim.stdout
    assert _report(lim.stdout) == _report(one.stdout)


def test_simulation_falls_back_to_more_shards(gossip, oracle):
    ev = _burst(gossip)
    sim = gossip.P2PGossipNetworkSimulation(N_BURST, topo_seed=8, options={"mem_limit": _budget(gossip, ev) << 20})
    sim.CreateRandomTopology(16.0 / (N_BURST - 1), 5.0)
    st = sim.Start(5.3, events=ev)
    assert sim.shards_used == 2
    a, b = sim.topology.links()
    r = oracle.run_oracle_b(N_BURST, 5_000_000, gossip.seconds_to_ns(5.2), a, b, ev["ns"], ev["node"],
                            ev["share_id"], threads=16)
    for k in STATS:
        assert np.array_equal(getattr(st, k), getattr(r, k)), k


def test_engine_reports_capacity_errors(gossip):
    # the budget is enforced: an engine that cannot hold its window fails cleanly with a
    # capacity code (what the callers above catch), never a fault
    n = 20000
    topo = gossip.Topology.gnp(n, 16.0 / (n - 1), 10, gossip.TOPO_SKIP)
    t_cut = gossip.seconds_to_ns(7.0)
    ev = gossip.make_schedule(n, 100, 5_000_000_000, t_cut)
    eng = gossip.Engine(n, 5_000_000, 5_000_000_000, t_cut)
    eng.set_option("mem_limit", 2 << 20)
    eng.set_topology(topo)
    with pytest.raises(gossip.GossipError) as ei:
        eng.set_schedule(ev)
        eng.run()
    assert ei.value.code in (gossip.E_CAPACITY, gossip.E_NOMEM)
    eng.close()
