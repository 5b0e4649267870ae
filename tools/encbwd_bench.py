"""Standalone timing of the deferred angle-encoder backward at C3 size (B = 256: ~16k line-graph
targets, ~2.03 M triplets, H = 4, L = 4, kin = 11): the fp32 VALU kernel and the bf16 matrix-core
kernel, HIP events around N launches each (tools/, not product code)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gnn-elasticity-predictor_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--targets", type=int, default=16020)
    ap.add_argument("--deg", type=int, default=126)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--b32", action="store_true", help="B = 32 size: 2,580 targets x ~98 in-edges")
    a = ap.parse_args()
    from alignn_mi355x import ops
    dev = "cuda"
    g = torch.Generator(device="cpu").manual_seed(0)
    if a.b32:
        a.targets, a.deg = 2580, 98
    n, H, L, kin, D = a.targets, 4, 4, 11, 256
    deg = torch.randint(a.deg // 2, a.deg * 3 // 2 + 1, (n,), generator=g)
    dst = torch.repeat_interleave(torch.arange(n), deg)
    src = torch.randint(0, n, (dst.numel(),), generator=g)
    csr = ops.GraphCSR(torch.stack([src, dst]).to(dev), n)
    T = dst.numel()
    xb = torch.randn(T, 12, device=dev)
    x = xb[:, :kin]
    W1 = torch.randn(D, kin, device=dev) * 0.5
    b1 = torch.randn(D, device=dev) * 0.5
    U = [torch.randn(n, H, D, device=dev) for _ in range(L)]
    Vd = [torch.randn(n, H, D, device=dev) for _ in range(L)]
    dz = [torch.randn(T, H, device=dev) for _ in range(L)]
    al = [torch.randn(T, H, device=dev) for _ in range(L)]
    f16 = torch.empty(T, D, dtype=torch.bfloat16, device=dev)
    ops.linear_smallk_bf16(x, W1, b1, f16, relu=True)
    dW1, db1 = torch.empty(D, kin, device=dev), torch.empty(D, device=dev)
    byt = 4.0 * (T * (kin + 1 + 2 * L * H) + 2 * L * n * H * D)
    for name, kw, extra in (("fp32 valu", {}, 0.0), ("bf16 mfma", {"F": f16}, 2.0 * T * D)):
        for _ in range(2):
            ops.enc_bwd(csr, x, W1, b1, U, Vd, dz, al, dW1, db1, **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            ops.enc_bwd(csr, x, W1, b1, U, Vd, dz, al, dW1, db1, **kw)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        print(f"{name}: T={T} n={n}  {us:8.1f} us/launch  {(byt + extra) / us / 1e6:6.2f} TB/s compulsory", flush=True)


if __name__ == "__main__":
    main()
