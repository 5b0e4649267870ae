"""Add (or refresh) one entry of profiles/pmc_dominant.json — the per-launch HBM traffic bench.py
reports as ``roofline.traffic`` — from a tools/pmc_traffic.py --json output.

usage: python tools/pmc_dominant_add.py TRAFFIC_JSON KEY KERNEL_SUBSTRING GRID "SOURCE TEXT"
KEY is the bench's probe key (e.g. "tconv_bwd_dst n15360 m184320"); the entry is the (kernel, grid)
row of TRAFFIC_JSON whose kernel name contains KERNEL_SUBSTRING."""
import json
import os
import sys

src, key, sub, grid, note = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5]
rows = [r for r in json.load(open(src)) if sub in r["kernel"] and r["grid"] == grid]
if len(rows) != 1:
    raise SystemExit(f"expected one row for {sub!r} grid {grid}, found {len(rows)}")
r = rows[0]
path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "pmc_dominant.json")
d = json.load(open(path))
d[key] = {"kernel": r["kernel"], "grid": grid, "launches": r["launches"], "fetch_bytes": round(r["fetch_bytes"]),
          "write_bytes": round(r["write_bytes"]), "traffic_bytes": round(r["traffic_bytes"]), "source": note}
json.dump(d, open(path, "w"), indent=1)
print(key, d[key]["traffic_bytes"])
