"""Dumps the line-graph attention kernels' outputs (lgconv.hip, forward + target-side backward) on
fixed seeded operands, so two library builds (ALIGNN_HIP_LIB) can be compared bitwise:
    python tools/lg3_dump.py OUT.pt            # with each build
    python tools/lg3_dump.py --compare A.pt B.pt
"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-elasticity-predictor_amd"))


def dump(path):
    from test_gpu_x_lg3 import DEGREES, _case, _run
    out = {}
    for H in (1, 2, 4):
        for drop in (0.0, 0.15):
            for degs in ("mp_mix", "ragged"):
                csr, m, t = _case(H, DEGREES[degs] * (3 if degs == "mp_mix" else 1), 11 + H, True)
                _, r = _run(csr, m, t, 256, H, drop, True)
                for k, v in r.items():
                    out[f"H{H}/p{drop}/{degs}/{k}"] = v.cpu()
    torch.save(out, path)
    print(f"{len(out)} tensors -> {path}")


def compare(a, b):
    A, B = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = [k for k in A if not torch.equal(A[k], B[k])]
    for k in bad[:20]:
        print("differs:", k, (A[k] - B[k]).abs().max().item())
    print(f"{len(A) - len(bad)}/{len(A)} bitwise equal")
    return 0 if not bad else 1


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        sys.exit(compare(sys.argv[2], sys.argv[3]))
    dump(sys.argv[1])
