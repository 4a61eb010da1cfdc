"""bench.py's N >= 2 path, as the driver launches it (torch.distributed.run, one process per rank,
`--gpus 2`), rehearsed on the one GPU of the test box: GOSSIP_DIST_BACKEND=gloo for the control
plane (RCCL refuses two ranks on one device) and GOSSIP_BENCH_NODES for a C4-shaped graph small
enough for two engines on one card.  The 2-rank line must count exactly the edge events and
generations of the N = 1 line (same shards: 2 in sequence on one GPU vs one per rank), with the
max-over-ranks timing, `n_gpus` = 2 and the whole-job value."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

NODES = "200000"
ARGS = ["--workload", "C4", "--steps", "4", "--warmup", "2", "--no-cpu-baseline", "--threads", "8"]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _line(cmd, env):
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_two_ranks_equal_one(tmp_path):
    env = dict(os.environ, GOSSIP_BENCH_NODES=NODES, GOSSIP_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    one = _line([sys.executable, "bench.py", "--gpus", "1"] + ARGS, env)
    two = _line([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                 "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2"] + ARGS,
                env)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert one["config"]["share_shards"] == two["config"]["share_shards"] == 2
    assert one["config"]["shards_per_gpu"] == 2 and two["config"]["shards_per_gpu"] == 1
    assert two["config"]["edge_events_timed"] == one["config"]["edge_events_timed"] > 0
    assert two["config"]["ticks_timed"] == one["config"]["ticks_timed"]
    v = two["config"]["edge_events_timed"] / (two["ms_per_step"] * two["steps"] / 1e3)
    assert abs(two["value"] - v) <= 1e-6 * v
    assert "REHEARSAL" in two["config"]["workload"]
