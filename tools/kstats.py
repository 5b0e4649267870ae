"""Per-step kernel time table from a rocprofv3 --stats kernel_stats.csv (steps = timed + warmup + probe)."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 14
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows) / 1e3 / steps
for r in rows[:top]:
    t = float(r["TotalDurationNs"]) / 1e3 / steps
    print(f"{t:8.1f} us/step {100 * t / tot:5.1f}%  calls/step={int(r['Calls']) / steps:6.1f} "
          f"avg={float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:90]}")
print(f"total kernel time per step {tot:.1f} us")
