"""Host cost of a replayed training step: wall time of trainer.step() calls issued back to back
(no synchronisation) against the device time of the same steps, at a bench configuration.  If the
host needs longer per step than the device, the device waits for the host's launches."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-elasticity-predictor_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(dev)
    tr = A.FusedTrainer(model, precision=a.precision)
    b = mp_like_batch(a.batch).to(dev)
    for i in range(3):
        tr.step(b, seed=i)
    tr.capture(b, mode="plan")
    for i in range(5):
        tr.step(b, seed=10 + i)
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for i in range(a.steps):
        h0 = time.perf_counter()
        tr.step(b, seed=100 + i)
        host.append(time.perf_counter() - h0)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"B={a.batch} {a.precision}: host per step {1e3 * sum(host) / len(host):.3f} ms "
          f"(min {1e3 * min(host):.3f}, max {1e3 * max(host):.3f}); issue loop {1e3 * (t1 - t0) / a.steps:.3f} ms/step; "
          f"device {1e3 * (t2 - t0) / a.steps:.3f} ms/step")


if __name__ == "__main__":
    main()
