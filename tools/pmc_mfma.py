"""Per-kernel MFMA counters from one rocprofv3 PMC pass:
    --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE

Per (kernel, grid) group, averaged over its dispatches:
  * mfma_gflop   = SQ_INSTS_VALU_MFMA_MOPS_F32 x 512 (rocprofv3's MfmaFlopsF32) — the matrix-core
                   work actually issued (compare with the GEMM's 2MNK);
  * busy_cycles  = SQ_VALU_MFMA_BUSY_CYCLES (summed over every SIMD: cycles an MFMA occupied one);
  * mfma_busy    = busy_cycles / (dispatch duration x 2.4 GHz x 1,024 SIMDs): the fraction of the
                   chip's matrix-core issue capacity the kernel kept busy (MI355X: 256 CUs x 4 SIMDs;
                   2.4 GHz peak clock, so a kernel under DVFS reads low, never high);
  * tflops       = mfma_gflop / duration.
Durations come from the same pass's dispatch timestamps (counter collection serialises kernels).

usage: python tools/pmc_mfma.py PMC_DIR [--json OUT] [--top N]
"""
import argparse
import collections
import csv
import glob
import json
import os

SIMDS = 256 * 4
CLOCK_HZ = 2.4e9


def load(d):
    path = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not path:
        raise SystemExit(f"no counter_collection.csv under {d}")
    disp = collections.defaultdict(dict)
    with open(path[0]) as f:
        for r in csv.DictReader(f):
            key = (r["Dispatch_Id"], r["Kernel_Name"], int(r["Grid_Size"]))
            disp[key][r["Counter_Name"]] = float(r["Counter_Value"])
            disp[key]["_dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    groups = collections.defaultdict(list)
    for (_, name, grid), c in disp.items():
        groups[(name, grid)].append(c)
    return groups


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--json")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = []
    for (name, grid), ds in load(a.pmc_dir).items():
        n = len(ds)
        dur = sum(c["_dur"] for c in ds) / n
        mops = sum(c.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0) for c in ds) / n
        busy = sum(c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for c in ds) / n
        if mops == 0 and busy == 0:
            continue
        rows.append({"kernel": name, "grid": grid, "launches": n, "avg_us_under_counters": dur * 1e6,
                     "mfma_gflop": mops * 512 / 1e9, "mfma_busy_cycles": busy,
                     "mfma_busy": busy / (dur * CLOCK_HZ * SIMDS) if dur > 0 else 0.0,
                     "tflops": mops * 512 / dur / 1e12 if dur > 0 else 0.0, "total_us": dur * 1e6 * n})
    rows.sort(key=lambda r: -r["total_us"])
    tot_t = sum(r["total_us"] for r in rows)
    tot_busy = sum(r["mfma_busy_cycles"] * r["launches"] for r in rows)
    for r in rows[: a.top]:
        print(f"{r['total_us']:9.0f}us n={r['launches']:4d} grid={r['grid']:8d} avg={r['avg_us_under_counters']:7.1f}us "
              f"{r['mfma_gflop']:7.3f} GF {r['tflops']:6.1f} TF/s busy={100 * r['mfma_busy']:5.1f}%  {r['kernel'][:80]}")
    if tot_t > 0:
        print(f"MFMA kernels: {tot_t:.0f} us in total, busy {100 * tot_busy / (tot_t * 1e-6 * CLOCK_HZ * SIMDS):.1f}% "
              f"of their matrix-core capacity")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
