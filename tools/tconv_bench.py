"""Microbenchmark of the attention kernels on the bench workload's graphs (B=32 MP-like, quirk and
fixed line-graph wiring): line graph (materialised features, with and without the dF rows; both
kernel families), atom graph.  Times each call with HIP events (median of R reps) on the current stream.

usage: python tools/tconv_bench.py [--reps 20] [--batch 32]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-elasticity-predictor_amd"))
from alignn_mi355x import ops  # noqa: E402
from alignn_mi355x.synthetic import mp_like_batch  # noqa: E402


def timeit(fn, reps):
    """Device time per call: ``reps`` calls captured in one HIP graph, replayed 3 times between two
    events; median replay / reps."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / reps)
    return sorted(ts)[1]


def run_graph(name, g, n, m, D, H, F, reps, out, nodf=False):
    dev = "cuda"
    # shapes the kernels assume (checked on the host before any launch)
    assert g.n == n and g.m == m, (g.n, n, g.m, m)
    assert F.size(0) >= m, (F.size(0), m)
    gen = torch.Generator(device=dev).manual_seed(0)
    r = lambda *s: torch.randn(*s, device=dev, generator=gen) * 0.5
    QKVR, U, Vd = r(n, 4 * D), r(n, H, D), r(n, H, D)
    wbar = r(D)
    aggV, S = torch.empty(n, D, device=dev), torch.empty(n, H, D, device=dev)
    sumA, mstat, den = (torch.empty(n, H, device=dev) for _ in range(3))
    dout, dq = r(n, D), torch.empty(n, D, device=dev)
    Sz, sigz = torch.empty(n, H, D, device=dev), torch.empty(n, H, device=dev)
    dz, al = torch.empty(max(m, 1), H, device=dev), torch.empty(max(m, 1), H, device=dev)
    dKV = torch.empty(n, 2 * D, device=dev)
    dF = None if nodf else torch.zeros_like(F)
    ops.tconv_fwd(g, D, H, QKVR, U, wbar, F, None, aggV, S, sumA, mstat, den, 0.15, 1)
    t_f = timeit(lambda: ops.tconv_fwd(g, D, H, QKVR, U, wbar, F, None, aggV, S, sumA, mstat, den, 0.15, 1), reps)
    t_b = timeit(lambda: ops.tconv_bwd_dst(g, D, H, QKVR, U, Vd, wbar, F, None, dout, aggV, mstat, den, dq, Sz,
                                           sigz, dz, al, dF, 0 if dF is None else 1, 0.15, 1), reps)
    t_s = timeit(lambda: ops.tconv_bwd_src(g, D, H, QKVR, dout, dz, al, dKV), reps)
    fam = g.family(D, H, F)
    res = {"fwd_us": t_f, "bwd_dst_us": t_b, "bwd_src_us": t_s, "n": n, "m": m, "family": fam}
    out[name] = res
    print(f"{name:28s} fam={fam} n={n:6d} m={m:7d}  fwd {t_f:8.1f} us  bwd_dst {t_b:8.1f} us  bwd_src {t_s:8.1f} us", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--json")
    a = ap.parse_args()
    D, H = 256, 4
    out = {}
    for lg_offset in ("num_nodes", "num_edges"):
        b = mp_like_batch(a.batch, lg_offset=lg_offset).to("cuda")
        E, T = b.edge_index.size(1), b.lg_edge_index.size(1)
        from alignn_mi355x.engine import BatchCache
        lg = BatchCache._line_graph(b.lg_edge_index, E, True)
        nl = lg.n  # line-graph nodes after compaction to the bonds with line-graph edges
        xa = torch.empty_like(b.lg_edge_attr)
        ops.gather_rows(b.lg_edge_attr, lg.perm_dst, xa)
        w1 = torch.randn(D, xa.size(1), device="cuda") * 0.3
        b1 = torch.randn(D, device="cuda") * 0.1
        F = torch.relu(xa @ w1.t() + b1)
        run_graph(f"line/{lg_offset}/F", lg, nl, T, D, H, F, a.reps, out)
        # the training step's configuration: materialised F, deferred encoder backward (no dF)
        for wave_items in (False, True):
            lg.policy = ops.SchedulePolicy(wave_items=wave_items)
            lg._sched = None
            run_graph(f"line/{lg_offset}/F/nodF/wi{int(wave_items)}", lg, nl, T, D, H, F, a.reps, out,
                      nodf=True)
        lg._sched = None
        if lg_offset == "num_nodes":
            N = b.x.size(0)
            ag = ops.GraphCSR(b.edge_index, N)
            Fe = torch.randn(E, D, device="cuda")
            run_graph("atom", ag, N, E, D, H, Fe, a.reps, out)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
