"""Standalone timing of the bf16-storage line-graph attention (alignn_lg_fwd_bf16 / _bwd_dst_bf16) on
the C3 line graph (B = 256 MP-like, PyG offset rule: 16,020 active bonds, 2,027,520 triplets), HIP
events around each call on the current stream (median of R reps), plus the max relative difference
to the fp32 single-wave kernels on the same bf16-representable rows.  The library is the in-tree
build unless ALIGNN_HIP_LIB names another (A/B builds).

usage: python tools/lgm_bench.py [--reps 20] [--batch 256] [--heads 4]
"""
import argparse
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "gnn-elasticity-predictor_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def timeit(fn, reps):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def rel(a, b):
    a, b = a.double(), b.double()
    d = torch.where(a == b, torch.zeros_like(a), a - b)
    fin = b[torch.isfinite(b)]
    return float(d.abs().max() / (fin.abs().max() if fin.numel() else torch.tensor(1.0)).clamp(min=1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--heads", type=int, default=4)
    ap.add_argument("--drop", type=float, default=0.15)
    a = ap.parse_args()
    from alignn_mi355x import ops
    from alignn_mi355x.engine import batch_cache
    from alignn_mi355x.synthetic import mp_like_batch
    bc = batch_cache(mp_like_batch(a.batch).to("cuda"))
    g = bc.lg
    n, m, D, H = g.n, g.m, 256, a.heads
    gen = torch.Generator(device="cuda").manual_seed(11)
    r = lambda *s: torch.randn(*s, device="cuda", generator=gen) * 0.5  # noqa: E731
    QKV = r(n, 3 * D)
    QKV[:, D:] = QKV[:, D:].bfloat16().float()
    U, Vd, dout, wbar = r(n, H, D), r(n, H, D), r(n, D), r(D)
    F16 = r(m, D).bfloat16()
    F = F16.float()
    KV16 = ops.cast_bf16(QKV[:, D:])
    outs, times = {}, {}
    for mode in ("fp32", "bf16"):
        outp, S = torch.empty(n, D, device="cuda"), torch.empty(n, H, D, device="cuda")
        sumA, mstat, den, sigz = (torch.empty(n, H, device="cuda") for _ in range(4))
        dq, Sz = torch.empty(n, D, device="cuda"), torch.empty(n, H, D, device="cuda")
        dz, al = torch.empty(m, H, device="cuda"), torch.empty(m, H, device="cuda")
        if mode == "fp32":
            fwd = lambda: ops.tconv_fwd(g, D, H, QKV, U, wbar, F, None, outp, S, sumA, mstat, den, a.drop, 9)  # noqa: E731
            bwd = lambda: ops.tconv_bwd_dst(g, D, H, QKV, U, Vd, wbar, F, None, dout, outp, mstat, den, dq, Sz, sigz,  # noqa: E731
                                            dz, al, None, 0, a.drop, 9)
        else:
            fwd = lambda: ops.lg_fwd_bf16(g, D, H, QKV, KV16, U, wbar, F16, outp, S, sumA, mstat, den, a.drop, 9)  # noqa: E731
            bwd = lambda: ops.lg_bwd_dst_bf16(g, D, H, QKV, KV16, U, Vd, wbar, F16, dout, outp, mstat, den, dq, Sz,  # noqa: E731
                                              sigz, dz, al, a.drop, 9)
        fwd()
        bwd()
        torch.cuda.synchronize()
        outs[mode] = dict(outp=outp.clone(), S=S.clone(), sumA=sumA.clone(), mstat=mstat.clone(), den=den.clone(),
                          dq=dq.clone(), Sz=Sz.clone(), sigz=sigz.clone(), dz=dz.clone(), al=al.clone())
        times[mode] = {"fwd_us": round(timeit(fwd, a.reps), 1), "bwd_dst_us": round(timeit(bwd, a.reps), 1)}
    fb = ops._lg_bf16_bytes(n, m, D, H, "fwd")
    bb = ops._lg_bf16_bytes(n, m, D, H, "bwd_dst")
    res = {"n": n, "m": m, "H": H, "lib": os.environ.get("ALIGNN_HIP_LIB", "in-tree"), "times": times,
           "bf16_fwd_TBps": round(fb / times["bf16"]["fwd_us"] * 1e-6, 3),
           "bf16_bwd_TBps": round(bb / times["bf16"]["bwd_dst_us"] * 1e-6, 3),
           "rel_diff_vs_fp32": {k: rel(outs["bf16"][k], outs["fp32"][k]) for k in outs["fp32"]}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
