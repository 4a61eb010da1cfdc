"""bench.py attaches committed PMC traffic (profiles/pmc_<workload>.json) to a line only when the
PMC pass ran the line's configuration -- the pull variant included (tile lists, early exit,
streams).  CPU only: the bench module is loaded, nothing is launched."""
import copy
import importlib.util
import json
import os

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _line_from_pmc(name):
    cfg = json.load(open(os.path.join(ROOT, "profiles", f"pmc_{name}.json")))["config"]
    line = {"n_gpus": 1, "warmup": cfg["warmup"], "steps": cfg["steps"],
            "config": {"live_words_per_node": cfg["live_words_per_node"]}}
    return line, dict(cfg["pull_variant"])


def test_pmc_traffic_attaches_only_to_its_own_variant():
    b = _bench()
    for name in ("C4", "C4_young"):
        line, variant = _line_from_pmc(name)
        t, why = b.pmc_traffic(name, line, variant)
        assert why is None and t > 1e10, (name, why)
        for key, other in (("pull_tiles", 1 - variant.get("pull_tiles", 0)), ("late_age", 0),
                           ("young_overlap", 0)):
            v2 = dict(variant, **{key: other})
            t2, why2 = b.pmc_traffic(name, line, v2)
            assert t2 is None and "pull_variant" in why2, (name, key)
        l2 = copy.deepcopy(line)
        l2["steps"] += 1
        assert b.pmc_traffic(name, l2, variant)[0] is None
        l3 = dict(line, n_gpus=2)
        assert b.pmc_traffic(name, l3, variant) == (None, "PMC pass is single-GPU")
