"""The recorded stream structure of a captured training step (alignn_plan_entries): every kernel
and cross-stream edge of the forward/backward plan in issue order, with its stream slot (0 = the
caller's stream, then the engine's side / aux streams in order of first use)."""
import argparse
import ctypes
import os
import re
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-elasticity-predictor_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--set", action="append", default=[], metavar="engine.ATTR=V")
    a = ap.parse_args()
    import alignn_mi355x as A
    from alignn_mi355x import _lib
    from alignn_mi355x.synthetic import mp_like_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(dev)
    for kv in a.set:
        k, v = kv.split("=", 1)
        setattr(model._engine, k.split(".", 1)[1], int(v))
    tr = A.FusedTrainer(model, precision=a.precision)
    b = mp_like_batch(a.batch).to(dev)
    tr.step(b, seed=1)
    tr.capture(b, mode="plan")
    lib = _lib.lib()
    for pi, plan in enumerate(tr._graph[3]):
        n = lib.alignn_plan_entries(plan, None, None, 0)
        kss = (ctypes.c_int32 * (3 * n))()
        names = (ctypes.c_char_p * n)()
        lib.alignn_plan_entries(plan, kss, names, n)
        print(f"== plan {pi}: {n} entries")
        for i in range(n):
            kind, slot, src = kss[3 * i], kss[3 * i + 1], kss[3 * i + 2]
            if kind == 0:
                nm = (names[i] or b"?").decode()
                nm = re.sub(r"^_ZN6alignn(3lg3)?\d+", "", nm)[:60]
                print(f"{i:4d} s{slot} {'    ' * slot}{nm}")
            elif kind == 1:
                print(f"{i:4d} s{slot} {'    ' * slot}<- wait s{src}")
    tr.release_capture()


if __name__ == "__main__":
    main()
