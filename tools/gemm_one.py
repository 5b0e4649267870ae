"""One GEMM shape issued R times (for per-launch PMC traffic of a single product, e.g. config C3's
dominant bf16 product over every bond: C[184320, 256] = A[184320, 256] . W^T).

usage: python tools/gemm_one.py --M 184320 --N 256 --K 256 [--bf16] [--reps 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-elasticity-predictor_amd"))
from alignn_mi355x import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=184320)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    A = torch.randn(a.M, a.K, device="cuda", generator=g)
    W = torch.randn(a.N, a.K, device="cuda", generator=g)
    b = torch.randn(a.N, device="cuda", generator=g)
    C = torch.empty(a.M, a.N, device="cuda")
    tile = ops.GEMM_BF16 if a.bf16 else 0
    path = ops.gemm(A, W.t(), C, bias=b, tile=tile, path_only=True)
    for _ in range(a.reps):
        ops.gemm(A, W.t(), C, bias=b, tile=tile)
    torch.cuda.synchronize()
    print(f"gemm M{a.M} N{a.N} K{a.K} {'bf16' if a.bf16 else 'fp32'}: path {path} ({'bf16 streaming' if path == 1 else 'tiled'}), "
          f"{a.reps} launches; algorithmic bytes per launch {4 * (a.M * a.K + a.N * a.K + a.M * a.N) / 1e6:.1f} MB")


if __name__ == "__main__":
    main()
