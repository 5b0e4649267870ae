"""Where does the step's wall time go? Host enqueue time vs device time, and the side stream's share.

For each configuration it times K steps of the bench workload (B=32, config C2) and prints
  host_ms  : time for the Python loop of K step() calls to return (no sync inside), per step
  wall_ms  : time until the device has finished them, per step
host ~= wall means the host cannot enqueue faster than the GPU drains (launch-bound).
Configurations: default eager; overlap off (everything on one stream); HIP-graph replay;
'drop-side' (timing diagnostic only, results are wrong): every launch inside the engine's side-stream
blocks is skipped, which bounds what perfect overlap of the weight-gradient work could give.

Usage: python tools/diag_overlap.py [--steps 20] [--batch 32]
"""
import argparse
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gnn-elasticity-predictor_amd"))


def build(batch_size, **engine_flags):
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    torch.manual_seed(1234)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).cuda()
    for k, v in engine_flags.items():
        setattr(model._engine, k, v)
    tr = A.FusedTrainer(model)
    b = mp_like_batch(batch_size).to("cuda")
    return tr, b


def timed(tr, b, steps, warm=5):
    for i in range(warm):
        tr.step(b, seed=i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        tr.step(b, seed=100 + i)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / steps * 1e3, (t2 - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=32)
    args = ap.parse_args()
    from alignn_mi355x import engine, ops

    res = {}
    tr, b = build(args.batch)
    eng = tr.model._engine
    print("engine flags:", {k: v for k, v in vars(eng).items() if isinstance(v, bool)})
    res["default"] = timed(tr, b, args.steps)
    eng.overlap = False
    res["overlap_off"] = timed(tr, b, args.steps)
    eng.overlap = True
    eng.defer_angle_bwd = not eng.defer_angle_bwd
    res["defer_angle_bwd=%d" % eng.defer_angle_bwd] = timed(tr, b, args.steps)
    eng.defer_angle_bwd = not eng.defer_angle_bwd
    # drop-side: skip every launch issued inside _side_work (wrong gradients; timing only)
    orig_enter, orig_exit = engine._side_work.__enter__, engine._side_work.__exit__
    real = {n: getattr(ops, n) for n in ("gemm", "colsum", "gemm_tn_smalln", "enc_bwd")}
    state = {"on": False}

    def wrap(fn):
        def f(*a, **k):
            if state["on"]:
                return a[2] if len(a) > 2 else None
            return fn(*a, **k)
        return f

    def enter(self):
        if self.side is not None:
            state["on"] = True
        return self

    def exit_(self, *exc):
        state["on"] = False
        return False

    for n, fn in real.items():
        setattr(ops, n, wrap(fn))
    engine._side_work.__enter__, engine._side_work.__exit__ = enter, exit_
    try:
        res["drop_side"] = timed(tr, b, args.steps)
    finally:
        for n, fn in real.items():
            setattr(ops, n, fn)
        engine._side_work.__enter__, engine._side_work.__exit__ = orig_enter, orig_exit
    for mode in ("plan", "graph"):
        tr.capture(b, mode=mode)
        res[mode] = timed(tr, b, args.steps)
        if mode == "plan":
            # host cost of one replay alone (device kept busy by a long queue, so no back-pressure)
            from alignn_mi355x import _lib
            plans = tr._graph[3]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                _lib.lib().alignn_plan_replay(plans[0], ops.stream_ptr())
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            print("plan replay host cost: %.3f ms per forward/backward plan" % ((t1 - t0) / args.steps * 1e3))
        tr.release_capture()
    for k, (h, w) in res.items():
        print(f"{k:12s} host {h:7.3f} ms/step   wall {w:7.3f} ms/step   {args.batch / w * 1e3:8.1f} graphs/s")


if __name__ == "__main__":
    main()
