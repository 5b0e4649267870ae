"""Standalone runs of the C2 step's dominant GEMM family (M 23,040 x 256 x 256 fp32: the line blocks'
skip projection A.W^T + bias, and its dX = dR.W product with beta = 1) for counter passes and A/B
timing: HIP events around R back-to-back calls (median per call), the same product through
torch.matmul (hipBLASLt) beside it, and optionally forced plans (--tile bits of AlignnGemmArgs.tile).

usage: python tools/gemm_probe.py [--iters 50] [--tile 0] [--which both|fwd|dx] [--M 23040] [--bf16]
"""
import argparse
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "gnn-elasticity-predictor_amd"))

import torch  # noqa: E402


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--which", default="both", choices=["both", "fwd", "dx"])
    ap.add_argument("--M", type=int, default=23040)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--bf16", action="store_true", help="bf16 matrix-core arithmetic")
    ap.add_argument("--no-lib", action="store_true")
    ap.add_argument("--io16", action="store_true", help="bf16 storage: A and (fwd) C bf16, dx with a bf16 dR")
    a = ap.parse_args()
    from alignn_mi355x import ops
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.randn(a.M, a.K, device="cuda", generator=g)
    W = torch.randn(a.N, a.K, device="cuda", generator=g) * 0.05
    bias = torch.randn(a.N, device="cuda", generator=g)
    dR = torch.randn(a.M, a.N, device="cuda", generator=g)
    Wd = torch.randn(a.N, a.K, device="cuda", generator=g) * 0.05   # dX = dR W (W [N, K] as [k, n] = [N, K])
    C1 = torch.empty(a.M, a.N, device="cuda")
    C2 = torch.randn(a.M, a.K, device="cuda", generator=g)
    if a.io16:
        X, C1, dR = X.bfloat16(), C1.bfloat16(), dR.bfloat16()
    res = {"M": a.M, "N": a.N, "K": a.K, "tile": a.tile, "bf16": a.bf16, "io16": a.io16}
    prec = "bf16" if a.bf16 else "fp32"
    flops = 2.0 * a.M * a.N * a.K
    with ops.gemm_precision(prec):
        if a.which in ("both", "fwd"):
            t = timeit(lambda: ops.gemm(X, W.t(), C1, bias=bias, tile=a.tile), a.iters)
            res["fwd_us"], res["fwd_tflops"] = t, round(flops / t / 1e6, 1)
        if a.which in ("both", "dx"):
            t = timeit(lambda: ops.gemm(dR, Wd, C2, beta=1.0, tile=a.tile), a.iters)
            res["dx_us"], res["dx_tflops"] = t, round(flops / t / 1e6, 1)
    if not a.no_lib:
        if a.bf16:
            Xb, Wb = X.bfloat16(), W.bfloat16()   # (bf16 in and out: half the bytes of fp32 storage)
            res["lib_fwd_us"] = timeit(lambda: torch.addmm(bias.bfloat16(), Xb, Wb.t()), a.iters)
            dRb, Wdb = dR.bfloat16(), Wd.bfloat16()
            res["lib_dx_us"] = timeit(lambda: torch.matmul(dRb, Wdb), a.iters)
        else:
            res["lib_fwd_us"] = timeit(lambda: torch.addmm(bias, X, W.t()), a.iters)
            res["lib_dx_us"] = timeit(lambda: torch.matmul(dR, Wd), a.iters)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
