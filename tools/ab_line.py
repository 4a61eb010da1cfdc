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
        parts.append(f"peer_rows {br['peer_rows'] / 1e9:.1f} GB")
print(" | ".join(parts), flush=True)
