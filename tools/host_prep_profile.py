"""Where the end-to-end loop's host time goes (config C5: B = 256 bf16 over an HBM-resident store).

Runs bench.end_to_end's loop by hand: per step, the captured plan is re-bound and replayed
(trainer.step) and the next batch is collated + prepared on a loader stream.  Reports the host time
of each phase of the preparation (collate, line-graph compaction / CSR, schedules) and a cProfile
of the preparation's functions.  Usage: python tools/host_prep_profile.py [--graphs 2000] [--steps 30]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gnn-elasticity-predictor_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", type=int, default=2000)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    import alignn_mi355x as A
    from alignn_mi355x import engine
    from alignn_mi355x.data import Data
    from alignn_mi355x.store import GraphStore
    from alignn_mi355x.synthetic import mp_like_graph

    dev = torch.device("cuda", 0)
    keys = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y")
    store = GraphStore.from_data_list([Data(**{k: getattr(mp_like_graph(g), k) for k in keys})
                                       for g in range(a.graphs)], dev)
    torch.manual_seed(0)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(dev)
    tr = A.FusedTrainer(model, precision="bf16")
    rng = np.random.default_rng(5)
    loader = torch.cuda.Stream(device=dev, priority=-1)
    phase = {"collate": 0.0, "cache": 0.0, "schedules": 0.0, "tensors": 0.0}

    def make(timed=False):
        t0 = time.perf_counter()
        with torch.cuda.stream(loader):
            b = store.collate(rng.choice(store.num_graphs, size=a.batch, replace=False), lg_offset="num_nodes")
            t1 = time.perf_counter()
            bc = engine.batch_cache(b, True)
            t2 = time.perf_counter()
            bc.schedules()
            t3 = time.perf_counter()
            bc.device_tensors()
            t4 = time.perf_counter()
        ev = torch.cuda.Event()
        ev.record(loader)
        b._alignn_ready = ev
        b._alignn_adopted = {loader.cuda_stream}
        if timed:
            for k, d in zip(phase, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
                phase[k] += d
        return b

    first = make()
    tr.capture(first)
    nxt = make()
    for i in range(5):
        tr.step(nxt, seed=i)
        nxt = make()
    torch.cuda.synchronize()

    # 1) phases with the step running concurrently (the real loop)
    t0 = time.perf_counter()
    hs = hm = 0.0
    for i in range(a.steps):
        cur = nxt
        ta = time.perf_counter()
        tr.step(cur, seed=100 + i)
        tb = time.perf_counter()
        nxt = make(timed=True)
        hs += tb - ta
        hm += time.perf_counter() - tb
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"loop: {dt / a.steps * 1e3:.3f} ms/step ({a.batch * a.steps / dt:.1f} graphs/s); host step "
          f"{hs / a.steps * 1e3:.3f} ms, host make {hm / a.steps * 1e3:.3f} ms", flush=True)
    print("make phases (ms/step): " + ", ".join(f"{k} {v / a.steps * 1e3:.3f}" for k, v in phase.items()), flush=True)

    # 2) the same with the GPU idle (preparation alone: host work + its own syncs)
    for k in phase:
        phase[k] = 0.0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        make(timed=True)
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"idle GPU: make+sync {dt / a.steps * 1e3:.3f} ms; phases: "
          + ", ".join(f"{k} {v / a.steps * 1e3:.3f}" for k, v in phase.items()), flush=True)

    # 3) bare step (pre-collated batch, no preparation in the loop)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        tr.step(nxt, seed=500 + i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"bare replay of one batch: {dt / a.steps * 1e3:.3f} ms/step", flush=True)

    # 4) cProfile of the preparation inside the loop
    pr = cProfile.Profile()
    for i in range(a.steps):
        cur = nxt
        tr.step(cur, seed=900 + i)
        pr.enable()
        nxt = make()
        pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
