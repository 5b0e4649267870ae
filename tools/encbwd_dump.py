"""Dumps the deferred angle-encoder backward's outputs (encbwd.hip) on fixed seeded operands, so two
library builds (ALIGNN_HIP_LIB) can be compared bitwise:
    python tools/encbwd_dump.py OUT.pt ; python tools/lg3_dump.py --compare A.pt B.pt
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-elasticity-predictor_amd"))


def main(path):
    from alignn_mi355x import ops
    out = {}
    for H, L, kin, D in ((4, 4, 11, 256), (2, 2, 7, 64), (1, 1, 16, 32)):
        g = torch.Generator().manual_seed(100 + H * L)
        n = 300
        degs = torch.randint(0, 40, (n,), generator=g)
        dst = torch.repeat_interleave(torch.arange(n), degs)
        src = torch.randint(0, n, (dst.numel(),), generator=g)
        csr = ops.GraphCSR(torch.stack([src, dst]).cuda(), n)
        T = dst.numel()
        r = lambda *s: torch.randn(*s, generator=g).cuda()  # noqa: E731
        x = r(T, kin)
        W1, b1 = r(D, kin) * 0.3, r(D) * 0.1
        Us = [r(n, H, D) for _ in range(L)]
        Vds = [r(n, H, D) for _ in range(L)]
        dzs = [r(T, H) for _ in range(L)]
        als = [r(T, H) for _ in range(L)]
        dW1, db1 = torch.empty(D, kin, device="cuda"), torch.empty(D, device="cuda")
        ops.enc_bwd(csr, x, W1, b1, Us, Vds, dzs, als, dW1, db1)
        torch.cuda.synchronize()
        out[f"H{H}L{L}k{kin}D{D}/dW1"] = dW1.cpu()
        out[f"H{H}L{L}k{kin}D{D}/db1"] = db1.cpu()
    torch.save(out, path)
    print(f"{len(out)} tensors -> {path}")


if __name__ == "__main__":
    main(sys.argv[1])
