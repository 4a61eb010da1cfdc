#!/usr/bin/env python3
"""The CLI capacity fallback of tests/test_shards_gpu.py::test_cli_falls_back_to_more_shards, with
its stderr shown: 4,096 distinct shares born in one tick of a 20,000-node graph under a 40 MB
budget (GPU box only)."""
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "p2p-gossip-simulation-ns3_amd"))
import gossip  # noqa: E402

N = 20000
rng = np.random.Generator(np.random.Philox(11))
nodes = rng.choice(N, size=4096, replace=False)
ev = gossip.events_from_arrays(5_000_001_000 + np.arange(4096, dtype=np.int64), nodes,
                               np.arange(1, 4097, dtype=np.uint32))
with tempfile.TemporaryDirectory() as d:
    evf = os.path.join(d, "ev.txt")
    np.savetxt(evf, np.stack([ev["ns"], ev["node"], ev["share_id"]], 1), fmt="%d")
    sim = os.path.join(ROOT, "p2p-gossip-simulation-ns3_amd", "lib", "gossip_sim")
    base = [f"--numNodes={N}", f"--connectionProb={16.0 / (N - 1)}", "--simTime=5.3", "--seed=8",
            f"--events={evf}", "--quiet"]
    for extra in ([], ["--memLimitMB=40"], ["--memLimitMB=40", "--shards=2"]):
        p = subprocess.run([sim, *base, *extra], capture_output=True, text=True, timeout=300)
        print("args", extra, "rc", p.returncode)
        print(" stderr:", p.stderr.strip().replace("\n", "\n         "))
        print(" engines:", [ln for ln in p.stdout.splitlines() if ln.startswith("engines")])
