"""Generate the committed golden fixtures under tests/golden/ from ORACLE A.

The reference has no tests, fixtures or golden logs and cannot run here (NS-3 is absent), so
these fixtures are the oracle's outputs for fixed seeds: regression pins for the oracle
(tests/test_golden.py) and parity targets for the HIP engine (tests/test_engine_gpu.py).
Run from the repo root:  python tests/golden/make_golden.py [case ...]
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.dirname(HERE))
import oracle  # noqa: E402
from golden_util import links_digest  # noqa: E402

CASES = {
    "c1_seed1": dict(num_nodes=10, connection_prob=0.3, sim_time_s=60.0, latency_ms=5.0, topo_seed=1, node_seed=1000),
    "c1_seed2": dict(num_nodes=10, connection_prob=0.3, sim_time_s=60.0, latency_ms=5.0, topo_seed=2, node_seed=2000),
    "c1_seed3": dict(num_nodes=10, connection_prob=0.3, sim_time_s=60.0, latency_ms=5.0, topo_seed=3, node_seed=3000),
    "n254_p03": dict(num_nodes=254, connection_prob=0.3, sim_time_s=60.0, latency_ms=5.0, topo_seed=4, node_seed=4000),
    "n300_collide": dict(num_nodes=300, connection_prob=0.05, sim_time_s=30.0, latency_ms=5.0, topo_seed=5, node_seed=5000, id_mask=0xFFF),
    "n60_lat37": dict(num_nodes=60, connection_prob=0.1, sim_time_s=20.05, latency_ms=3.7, topo_seed=6, node_seed=6000),
    "n120_sparse_lat1": dict(num_nodes=120, connection_prob=0.02, sim_time_s=12.0, latency_ms=1.0, topo_seed=7, node_seed=7000),
    # 4096-node short windows, sparse (avg degree ~12) and dense (C2's p = 0.3)
    "n4096_sparse_short": dict(num_nodes=4096, connection_prob=0.003, sim_time_s=5.5, latency_ms=5.0, topo_seed=8, node_seed=8000),
    "n4096_p03_short": dict(num_nodes=4096, connection_prob=0.3, sim_time_s=5.12, latency_ms=5.0, topo_seed=9, node_seed=9000),
}


def only(names):
    return {k: v for k, v in CASES.items() if k in names} if names else CASES


def links_fields(a, b):
    # large link sets (the dense 4096-node case has 2.5M keys) are pinned by a digest
    if a.size <= 100_000:
        return dict(link_a=a, link_b=b)
    return dict(link_count=np.array(a.size, np.uint64), link_sha256=np.array(links_digest(a, b)))


def main():
    for name, kw in only(sys.argv[1:]).items():
        r = oracle.run_reference(**kw)
        per = np.array(r.periodic, dtype=np.int64).reshape(-1, 4)
        np.savez_compressed(
            os.path.join(HERE, name + ".npz"),
            params=np.array(json.dumps(kw)),
            gen=r.gen, recv=r.recv, fwd=r.fwd, sent=r.sent, processed=r.processed,
            peers=r.peers, sockets=r.sockets, periodic=per,
            **links_fields(r.links[0], r.links[1]),
            edge_events=np.array(r.edge_events, np.uint64))
        print(f"{name}: edge events {r.edge_events}, gens {int(r.gen.sum())}, wall {r.wall_s:.2f}s")


if __name__ == "__main__":
    main()
