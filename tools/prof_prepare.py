"""Host-side profile of the end-to-end loop (store collate + batch preparation + re-bound step): where
the per-step host time goes.  cProfile over `steps` iterations of bench.end_to_end's loop body.

usage: python tools/prof_prepare.py [--batch 32] [--graphs 2000] [--steps 30] [--variable]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "gnn-elasticity-predictor_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--graphs", type=int, default=2000)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--variable", action="store_true")
    ap.add_argument("--precision", default="fp32")
    a = ap.parse_args()
    import alignn_mi355x as A
    from alignn_mi355x.data import Data
    from alignn_mi355x.engine import prepare_batch
    from alignn_mi355x.store import GraphStore
    from alignn_mi355x.synthetic import mp_like_graph, variable_mp_like_graph
    keys = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y")
    gen = variable_mp_like_graph if a.variable else mp_like_graph
    st = GraphStore.from_data_list([Data(**{k: getattr(gen(g), k) for k in keys}) for g in range(a.graphs)], "cuda")
    cap = st.capacity(a.batch) if a.variable else None
    torch.manual_seed(0)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).cuda()
    tr = A.FusedTrainer(model, precision=a.precision)
    rng = np.random.default_rng(0)
    first = next(i for i in (rng.choice(st.num_graphs, a.batch, replace=False) for _ in range(1000))
                 if cap is None or st.fits(i, cap) is not None)
    tr.capture(st.collate(first, capacity=cap))
    loader = torch.cuda.Stream(priority=-1 if a.batch >= 128 else 0)

    def make():
        with torch.cuda.stream(loader):
            b = st.collate(rng.choice(st.num_graphs, size=a.batch, replace=False), capacity=cap)
        prepare_batch(b, loader)
        return b

    nxt = make()
    for i in range(5):
        tr.step(nxt, seed=i)
        nxt = make()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t_step = t_make = 0.0
    t0 = time.perf_counter()
    pr.enable()
    for i in range(a.steps):
        ta = time.perf_counter()
        tr.step(nxt, seed=100 + i)
        tb = time.perf_counter()
        nxt = make()
        t_step += tb - ta
        t_make += time.perf_counter() - tb
    pr.disable()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"B={a.batch} variable={a.variable}: {a.batch * a.steps / dt:.1f} graphs/s, host ms/step: step "
          f"{t_step / a.steps * 1e3:.3f}, make {t_make / a.steps * 1e3:.3f}; rebinds {tr.rebinds} misses "
          f"{tr.rebind_misses}")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(45)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
    print(s.getvalue())


if __name__ == "__main__":
    main()
