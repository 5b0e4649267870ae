"""Step timeline from a rocprofv3 kernel trace: busy union, per-queue busy time, idle gaps.

Steps are delimited by the AdamW kernel (one per step).  Prints, for one full step (the last by default), the
device-busy union, each queue's busy time, and the largest gaps where no kernel runs at all, with
the kernels either side — launch gaps on the critical path show up there.

Usage: python tools/timeline.py gpurun_out/rocprof/run_kernel_trace.csv [--top 15]
"""
import argparse
import csv
import re


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name.replace("void ", "").replace("alignn::", "")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--by-kernel", action="store_true", help="per-queue time by kernel (name, grid) in the step")
    ap.add_argument("--sequence", action="store_true", help="every kernel of the step in start order")
    ap.add_argument("--step", type=int, default=1,
                    help="which step, counted from the end (1: the last; bench.py's serialized roofline "
                         "replays are its last 3 steps, so 4+ is a timed, concurrent one)")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                         r["Kernel_Name"] + (f" grid={int(r['Grid_Size_X']) * int(r['Grid_Size_Y']) * int(r['Grid_Size_Z'])}" if a.by_kernel else "")))
    rows.sort()
    ends = [e for s, e, q, n in rows if "adamw_kernel" in n]
    if len(ends) < a.step + 2:
        raise SystemExit(f"need at least {a.step + 2} steps in the trace")
    t0, t1 = ends[-a.step - 1], ends[-a.step]
    ks = [r for r in rows if r[0] >= t0 and r[1] <= t1]
    span = (t1 - t0) / 1e3
    busy, gaps, cur_s, cur_e, prev = 0, [], None, None, None
    for s, e, q, n in ks:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, prev, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        prev = n if e >= (cur_e or 0) else prev
    busy += cur_e - cur_s
    per_q = {}
    for s, e, q, n in ks:
        per_q[q] = per_q.get(q, 0) + (e - s)
    print(f"step {span:.1f} us, {len(ks)} kernels, device busy (union) {busy/1e3:.1f} us, "
          f"idle {span - busy/1e3:.1f} us in {len(gaps)} gaps")
    for q, t in sorted(per_q.items()):
        nq = sum(1 for r in ks if r[2] == q)
        print(f"  queue {q}: {nq} kernels, busy {t/1e3:.1f} us")
    gaps.sort(reverse=True)
    hist = {}
    for g, _, _ in gaps:
        b = min(int(g / 1e3), 20)
        hist[b] = hist.get(b, 0) + g
    print("idle by gap length (us bucket: total us): " +
          ", ".join(f"{b}: {t/1e3:.0f}" for b, t in sorted(hist.items())))
    for g, p, n in gaps[:a.top]:
        print(f"  gap {g/1e3:7.1f} us  after {short(p)}  before {short(n)}")
    if a.by_kernel:
        for q in sorted(per_q):
            agg = {}
            for s_, e_, q_, n in ks:
                if q_ == q:
                    k = short(n) + " " + n.split(" grid=")[-1]
                    c, t = agg.get(k, (0, 0))
                    agg[k] = (c + 1, t + e_ - s_)
            print(f"queue {q} by kernel:")
            for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:a.top * 2]:
                print(f"  {t/1e3:8.1f} us  n={c:3d}  {k}")
    if a.sequence:
        # every kernel of the step in start order: queue, start and end (us from the step start)
        print("sequence (queue, start, end, duration us):")
        for s, e, q, n in ks:
            print(f"  q{q} {(s - t0)/1e3:8.1f} {(e - t0)/1e3:8.1f} {(e - s)/1e3:7.1f}  {short(n)}")


if __name__ == "__main__":
    main()
