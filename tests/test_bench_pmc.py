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


def test_pmc_traffic_keys_every_launch_option_and_the_build():
    # the options that shape the launches (young grid, caps, ages ...) and the library build are
    # part of the match key: a pass of another build or another k_pull_young grid never attaches
    b = _bench()
    line, variant = _line_from_pmc("C4_young")
    variant = dict(variant, options={k: 0 for k in b.LAUNCH_OPTIONS}, young_grid_blocks=32768,
                   lib_sha256="0123456789abcdef")
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "profiles")
        os.makedirs(path)
        cfg = {"workload": "C4", "warmup": line["warmup"], "steps": line["steps"],
               "live_words_per_node": line["config"]["live_words_per_node"], "pull_variant": variant}
        with open(os.path.join(path, "pmc_C4_young.json"), "w") as f:
            json.dump({"hbm_bytes_per_launch": 4.9e10, "config": cfg}, f)
        root = b.ROOT
        b.ROOT = d
        try:
            assert b.pmc_traffic("C4_young", line, variant) == (4.9e10, None)
            for change in ({"young_grid_blocks": 16384}, {"lib_sha256": "fedcba9876543210"},
                           {"options": dict(variant["options"], young_cap=8)},
                           {"options": dict(variant["options"], young_list_cap=64)},
                           {"options": dict(variant["options"], young_age=4)}):
                t, why = b.pmc_traffic("C4_young", line, dict(variant, **change))
                assert t is None and "pull_variant" in why, change
        finally:
            b.ROOT = root


def test_young_breakdown_adds_up_to_the_engine_count():
    # young_bytes_moved restated from engine.hip (gossip_engine_get_counters): 128 B per slot line
    # read, fallback row, dense row written, slot line written, unhinted second line, list line and
    # seen row written whole; 5 B per peer id + hint; 8 B per own seen word read / written; per
    # launch 8 (n + 1) + 16 n of row pointers and counters
    import random
    b = _bench()
    rnd = random.Random(5)
    for _ in range(20):
        n = rnd.randrange(1, 10_000_000)
        yl = rnd.randrange(1, 50)
        acc = {k: rnd.randrange(0, 10**9) for k in ("young_sl", "young_fb", "young_col_ids", "young_seen_reads",
                                                     "young_seen_writes", "young_rows_written", "young_slot_writes",
                                                     "young_line2_misses", "young_fresh_lines", "young_list_lines")}
        engine = (128 * (acc["young_sl"] + acc["young_fb"] + acc["young_rows_written"] + acc["young_slot_writes"] +
                         acc["young_line2_misses"] + acc["young_list_lines"] + acc["young_fresh_lines"]) +
                  5 * acc["young_col_ids"] + 8 * (acc["young_seen_reads"] + acc["young_seen_writes"]) +
                  yl * (8 * (n + 1) + 16 * n))
        bd = b.young_breakdown(acc, yl, n)
        assert abs(sum(bd.values()) - engine / yl) <= 1e-9 * engine / yl
