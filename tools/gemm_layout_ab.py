"""Standalone timing of the M 23,040 x 256 x 256 products of the B = 32 step by operand layout:
A.W^T (B K-contiguous, the forward skip projection), dX += dR.W (B N-contiguous, beta = 1, the
backward), and the same dX product through a transposed weight copy (B K-contiguous, beta = 1).

usage: python tools/gemm_layout_ab.py [--reps 50]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-elasticity-predictor_amd"))
from alignn_mi355x import ops  # noqa: E402


def timed(fn, reps):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    M, D = 23040, 256
    g = torch.Generator(device="cuda").manual_seed(0)
    X = torch.randn(M, D, device="cuda", generator=g)
    W = torch.randn(D, D, device="cuda", generator=g)      # [out, in]
    Wt = W.t().contiguous()                                  # [in, out]
    b = torch.randn(D, device="cuda", generator=g)
    C = torch.empty(M, D, device="cuda")
    dX = torch.randn(M, D, device="cuda", generator=g)
    dX2 = dX.clone()
    print(f"A.W^T + b      (B K-contig):        {timed(lambda: ops.gemm(X, W.t(), C, bias=b), a.reps):7.1f} us")
    print(f"dX += dR.W     (B N-contig, beta 1): {timed(lambda: ops.gemm(X, W, dX, beta=1.0), a.reps):7.1f} us")
    print(f"dX += dR.(Wt)^T (B K-contig, beta 1): {timed(lambda: ops.gemm(X, Wt.t(), dX2, beta=1.0), a.reps):7.1f} us")
    print(f"C = dR.W       (B N-contig, beta 0): {timed(lambda: ops.gemm(X, W, C), a.reps):7.1f} us")
    r1 = torch.empty(M, D, device="cuda")
    r2 = torch.empty(M, D, device="cuda")
    ops.gemm(X, W, r1)
    ops.gemm(X, Wt.t(), r2)
    torch.cuda.synchronize()
    print("bitwise equal across layouts:", bool(torch.equal(r1, r2)))


if __name__ == "__main__":
    main()
