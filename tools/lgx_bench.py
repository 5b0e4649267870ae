"""Standalone timing of the line-graph attention with streamed edge-feature rows (the angle encoder's
hidden layer materialised by linear_smallk) against the recompute path (alignn_lg_fwd_x /
alignn_lg_bwd_dst_x: the rows recomputed from the 11 raw inputs on the matrix cores), fp32 (config
C2 wiring) and bf16 storage (config C3), on the MP-like line graph of B graphs (PyG offset rule).
HIP events around each call (median of R reps); also the deferred encoder backward (bf16: mask read
from the stored layer vs recomputed).  The library is the in-tree build unless ALIGNN_HIP_LIB names
another (A/B builds).

usage: python tools/lgx_bench.py [--reps 20] [--batch 32 256] [--only fwd_bf16_x bwd_bf16_x ...]
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
    return round(ts[len(ts) // 2], 1)


def one(B, reps, drop, only=None):
    from alignn_mi355x import ops
    from alignn_mi355x.engine import batch_cache
    from alignn_mi355x.synthetic import mp_like_batch
    bc = batch_cache(mp_like_batch(B).to("cuda"))
    g = bc.lg
    n, m, D, H, L = g.n, g.m, 256, 4, 4
    gen = torch.Generator(device="cuda").manual_seed(11)
    r = lambda *s: torch.randn(*s, device="cuda", generator=gen) * 0.5  # noqa: E731
    QKV, U, Vd, dout, wbar = r(n, 3 * D), r(n, H, D), r(n, H, D), r(n, D), r(D)
    x = bc.xa
    W1, b1 = (r(D, 11) * 0.6).contiguous(), r(D) * 0.2
    KV16 = ops.cast_bf16(QKV)[:, D:]
    F, F16 = torch.empty(m, D, device="cuda"), torch.empty(m, D, device="cuda", dtype=torch.bfloat16)
    res = {"B": B, "n": n, "m": m}
    outp, S = torch.empty(n, D, device="cuda"), torch.empty(n, H, D, device="cuda")
    sumA, mstat, den, sigz = (torch.empty(n, H, device="cuda") for _ in range(4))
    dq, Sz = torch.empty(n, D, device="cuda"), torch.empty(n, H, D, device="cuda")
    dz, al = torch.empty(m, H, device="cuda"), torch.empty(m, H, device="cuda")
    calls = {
        "linear_smallk_f32": lambda: ops.linear_smallk(x, W1, b1, F, relu=True),
        "linear_smallk_bf16": lambda: ops.linear_smallk_bf16(x, W1, b1, F16, relu=True),
        "fwd_f32_rows": lambda: ops.tconv_fwd(g, D, H, QKV, U, wbar, F, None, outp, S, sumA, mstat, den, drop, 9),
        "fwd_f32_x": lambda: ops.lg_fwd_x(g, D, H, QKV, None, U, wbar, x, W1, b1, outp, S, sumA, mstat, den, drop, 9),
        "bwd_f32_rows": lambda: ops.tconv_bwd_dst(g, D, H, QKV, U, Vd, wbar, F, None, dout, outp, mstat, den, dq, Sz,
                                                  sigz, dz, al, None, 0, drop, 9),
        "bwd_f32_x": lambda: ops.lg_bwd_dst_x(g, D, H, QKV, None, U, Vd, wbar, x, W1, b1, dout, outp, mstat, den, dq,
                                              Sz, sigz, dz, al, drop, 9),
        "fwd_bf16_rows": lambda: ops.lg_fwd_bf16(g, D, H, QKV, KV16, U, wbar, F16, outp, S, sumA, mstat, den, drop, 9),
        "fwd_bf16_x": lambda: ops.lg_fwd_x(g, D, H, QKV, KV16, U, wbar, x, W1, b1, outp, S, sumA, mstat, den, drop,
                                           9),
        "bwd_bf16_rows": lambda: ops.lg_bwd_dst_bf16(g, D, H, QKV, KV16, U, Vd, wbar, F16, dout, outp, mstat, den, dq,
                                                     Sz, sigz, dz, al, drop, 9),
        "bwd_bf16_x": lambda: ops.lg_bwd_dst_x(g, D, H, QKV, KV16, U, Vd, wbar, x, W1, b1, dout, outp, mstat, den, dq,
                                               Sz, sigz, dz, al, drop, 9),
    }
    Us, Vds = [r(n, H, D) for _ in range(L)], [r(n, H, D) for _ in range(L)]
    dzs, als = [r(m, H) for _ in range(L)], [r(m, H) for _ in range(L)]
    dW1, db1 = torch.empty(D, 11, device="cuda"), torch.empty(D, device="cuda")
    calls["enc_bwd_f32"] = lambda: ops.enc_bwd(g, x, W1, b1, Us, Vds, dzs, als, dW1, db1)
    calls["enc_bwd_bf16_rows"] = lambda: ops.enc_bwd(g, x, W1, b1, Us, Vds, dzs, als, dW1, db1, F=F16)
    calls["enc_bwd_bf16_x"] = lambda: ops.enc_bwd(g, x, W1, b1, Us, Vds, dzs, als, dW1, db1, bf16=True)
    if only:
        calls = {k: v for k, v in calls.items() if k in only}
    for k, fn in calls.items():
        fn()
        torch.cuda.synchronize()
    for k, fn in calls.items():
        res[k + "_us"] = timeit(fn, reps)
    if only:
        return res
    for kind, p in (("f32", 4), ("bf16", 2)):
        fr, fx = ops._tconv_bytes(n, m, D, H, "fwd", 0, f_elem=p), ops._lg_x_bytes(n, m, D, H, "fwd", p)
        br, bx = ops._tconv_bytes(n, m, D, H, "bwd_dst", 0, f_elem=p), ops._lg_x_bytes(n, m, D, H, "bwd_dst", p)
        res[f"mbyte_fwd_{kind}_rows_vs_x"] = [round(fr / 1e6, 1), round(fx / 1e6, 1)]
        res[f"mbyte_bwd_{kind}_rows_vs_x"] = [round(br / 1e6, 1), round(bx / 1e6, 1)]
    res["per_layer_f32_rows_vs_x_us"] = [round(res["fwd_f32_rows_us"] + res["bwd_f32_rows_us"], 1),
                                         round(res["fwd_f32_x_us"] + res["bwd_f32_x_us"], 1)]
    res["per_layer_bf16_rows_vs_x_us"] = [round(res["fwd_bf16_rows_us"] + res["bwd_bf16_rows_us"], 1),
                                          round(res["fwd_bf16_x_us"] + res["bwd_bf16_x_us"], 1)]
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, nargs="+", default=[32, 256])
    ap.add_argument("--drop", type=float, default=0.15)
    ap.add_argument("--only", nargs="+", help="time only these calls (e.g. fwd_bf16_x bwd_bf16_x)")
    a = ap.parse_args()
    for B in a.batch:
        print(json.dumps({"lib": os.environ.get("ALIGNN_HIP_LIB", "in-tree"), **one(B, a.reps, a.drop, a.only)}),
              flush=True)


if __name__ == "__main__":
    main()
