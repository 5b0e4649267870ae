"""Average duration per (kernel, grid size) from a rocprofv3 --kernel-trace CSV: separates the
launches of one kernel template on different graphs (e.g. line graph vs atom graph), which
--stats merges.  usage: python tools/trace_by_grid.py run_kernel_trace.csv [filter]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
d = collections.defaultdict(list)
for r in rows:
    if flt in r["Kernel_Name"]:
        d[(r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"]))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (name, grid), v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v) / len(v):9.1f} us avg  n={len(v):5d}  grid={grid:9d}  {name}")
