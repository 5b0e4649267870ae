"""Per-kernel SQ instruction-mix / stall counters from one rocprofv3 PMC pass:
    --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
          SQ_INSTS_LDS SQ_INSTS_SALU

Per (kernel, grid) group, averaged over its dispatches (ratios of summed counters):
  * wait_any  = SQ_WAIT_ANY / SQ_WAVE_CYCLES       (wave cycles waiting on anything, memory included)
  * wait_dep  = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES  (wave cycles waiting for an instruction dependency)
  * valu_act  = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (wave cycles issuing VALU)
  * valu/lds/salu = instructions per dispatch (millions)

usage: python tools/pmc_sq.py PMC_DIR [--json OUT] [--top N]
"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--json")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.pmc_dir, "*counter_collection.csv"))
    if not path:
        raise SystemExit(f"no counter_collection.csv under {a.pmc_dir}")
    disp = collections.defaultdict(dict)
    with open(path[0]) as f:
        for r in csv.DictReader(f):
            key = (r["Dispatch_Id"], r["Kernel_Name"], int(r["Grid_Size"]))
            disp[key][r["Counter_Name"]] = float(r["Counter_Value"])
            disp[key]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    groups = collections.defaultdict(lambda: collections.Counter())
    counts = collections.Counter()
    for (_, name, grid), c in disp.items():
        groups[(name, grid)].update(c)
        counts[(name, grid)] += 1
    rows = []
    for key, c in groups.items():
        n = counts[key]
        wc = max(c.get("SQ_WAVE_CYCLES", 0.0), 1.0)
        rows.append({"kernel": key[0], "grid": key[1], "launches": n, "avg_us": c["_dur"] / n * 1e6,
                     "total_us": c["_dur"] * 1e6,
                     "wait_any": c.get("SQ_WAIT_ANY", 0) / wc, "wait_dep": c.get("SQ_WAIT_INST_ANY", 0) / wc,
                     "valu_act": c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
                     "valu_M": c.get("SQ_INSTS_VALU", 0) / n / 1e6, "lds_M": c.get("SQ_INSTS_LDS", 0) / n / 1e6,
                     "salu_M": c.get("SQ_INSTS_SALU", 0) / n / 1e6})
    rows.sort(key=lambda r: -r["total_us"])
    for r in rows[:a.top]:
        print(f"{r['total_us']:8.0f}us n={r['launches']:4d} avg={r['avg_us']:7.1f}us wait_any={r['wait_any']:.2f} "
              f"wait_dep={r['wait_dep']:.2f} valu_act={r['valu_act']:.2f} valu={r['valu_M']:7.2f}M "
              f"lds={r['lds_M']:6.2f}M salu={r['salu_M']:6.2f}M  {r['kernel'][:70]}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
