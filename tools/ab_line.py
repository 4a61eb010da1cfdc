"""One summary line of a bench.py JSON result (A/B scripts): value, ms/tick, per-kernel times/bytes."""
import json
import sys

name, path = sys.argv[1], sys.argv[2]
d = json.loads(open(path).read().strip().splitlines()[-1])
r = d["roofline"]
ks = r.get("kernels", {})
parts = [f"[{name}] value {d['value']:.4e} ms/step {d['ms_per_step']:.2f}",
         f"phase {r['avg_launch_ms']:.2f} ms {r['bytes_per_launch'] / 1e9:.1f} GB frac {r['frac']:.3f}"]
for k, v in ks.items():
    parts.append(f"{k} {v['avg_launch_ms']:.2f} ms {v['bytes_per_launch'] / 1e9:.1f} GB")
    br = v.get("bytes_breakdown_per_launch", {})
    if "peer_rows" in br:
        parts.append(f"peer_rows {br['peer_rows'] / 1e9:.1f} GB occ {br['peer_occupancy'] / 1e9:.2f} GB "
                     f"seen_rd {br['own_seen_read'] / 1e9:.1f} GB sat_skips {v.get('saturated_tiles_skipped_per_launch', 0) / 1e6:.1f}M "
                     f"dense_tiles {v.get('dense_row_tiles_last_tick', 0)} "
                     f"items {v.get('items_per_launch', 0) / 1e6:.1f}M gather {v.get('gather_items_per_launch', 0) / 1e6:.1f}M")
c = d["config"]
parts.append(f"words {c['live_words_per_node']}/{c['window_capacity_words']} early {c.get('window_early_retires')} "
             f"shards {c['share_shards']} retried {c.get('shards_retried')}")
print(" | ".join(parts), flush=True)
