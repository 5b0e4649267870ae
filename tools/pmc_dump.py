"""Every counter of one rocprofv3 PMC pass, per (kernel, grid) group, averaged per dispatch; SQ_* cycle
counters also as a fraction of SQ_WAVE_CYCLES when that counter is in the pass.

usage: python tools/pmc_dump.py PMC_DIR [--match SUBSTR] [--top N]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--match", default="")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.pmc_dir, "**", "*counter_collection.csv"), recursive=True)
    if not path:
        raise SystemExit(f"no counter_collection.csv under {a.pmc_dir}")
    disp = collections.defaultdict(dict)
    with open(path[0]) as f:
        for r in csv.DictReader(f):
            key = (r["Dispatch_Id"], r["Kernel_Name"], int(r["Grid_Size"]))
            disp[key][r["Counter_Name"]] = disp[key].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            disp[key]["_us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    groups = collections.defaultdict(collections.Counter)
    counts = collections.Counter()
    for (_, name, grid), c in disp.items():
        if a.match in name:
            groups[(name, grid)].update(c)
            counts[(name, grid)] += 1
    rows = sorted(groups.items(), key=lambda kv: -kv[1]["_us"])[:a.top]
    for (name, grid), c in rows:
        n = counts[(name, grid)]
        wc = c.get("SQ_WAVE_CYCLES")
        parts = []
        for k in sorted(c):
            if k == "_us":
                continue
            v = c[k] / n
            s = f"{k}={v:.4g}"
            if wc and k.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY")) and k != "SQ_WAVE_CYCLES":
                s += f"({c[k] / wc:.2f})"
            parts.append(s)
        print(f"{name[:90]} grid={grid} n={n} avg={c['_us'] / n:.1f}us\n    " + " ".join(parts))


if __name__ == "__main__":
    main()
