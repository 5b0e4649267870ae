"""Golden vectors for KNN density weighting from the reference's own
``compute_global_knn_weights`` (scripts/train.py:930-1010; sklearn NearestNeighbors path), run in the
build container with ``oracle/torch_geometric`` standing in for PyG (as make_golden.py).

Model: HeteroAlignnRegressor (MP-like dims, hidden 64, 4 heads, 2 layers, seed 21); 3 batches of 10
small MP-like graphs (20 atoms) with ``train_idx`` 100..129.  k = 20, eps 1e-6, alpha 0.75, beta 1e-4,
no clip, and clip [3.2, 3.8] (raw weights span 3.0-4.2)
(k, eps, alpha: the reference's defaults, train.py:1184-1189; beta and the clip range chosen so the
weights do not all land on a clip bound).  Output ``tests/golden/knn.npz``: ``in/b{i}/*``,
``m/*`` state dict, ``out/Z`` (model.embed per graph), ``out/idx`` / ``out/w`` (the weight map).

Run:  python tests/golden/make_golden_knn.py
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "gnn-elasticity-predictor_amd"))
sys.path.insert(0, "/root/reference")

import scripts.train as ref  # noqa: E402
from torch_geometric.data import Batch as ShimBatch, Data as ShimData  # noqa: E402

from alignn_mi355x.synthetic import mp_like_graph  # noqa: E402

KEYS = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y")
# beta scaled down: the reference feeds raw targets (1..300) into the local variance, which with
# beta 1 drives every weight onto the clip floor; these keep the weights spread (two clip settings)
KNN = dict(k=20, eps=1e-6, alpha=0.75, beta=1e-4, clip_min=None, clip_max=None)
KNN_CLIP = dict(KNN, clip_min=3.2, clip_max=3.8)


def main():
    batches = []
    for bi in range(3):
        ds = []
        for g in range(10):
            d = mp_like_graph(200 + 10 * bi + g, n_atoms=20, half_degree=3)
            sd = ShimData(**{k: getattr(d, k) for k in KEYS})
            sd.train_idx = torch.tensor([100 + 10 * bi + g])
            ds.append(sd)
        batches.append(ShimBatch.from_data_list(ds))
    torch.manual_seed(21)
    model = ref.HeteroAlignnRegressor(ref.AlignnRegressor(206, 36, 11, 289, 2, 64, 2, 4, 0.15), 2)
    wmap = ref.compute_global_knn_weights(model, batches, torch.device("cpu"), None, **KNN)
    wclip = ref.compute_global_knn_weights(model, batches, torch.device("cpu"), None, **KNN_CLIP)
    model.eval()
    with torch.no_grad():
        Z = torch.cat([model.embed(b) for b in batches])
    arrays = {"out/Z": Z.numpy(), "out/idx": np.asarray(sorted(wmap), dtype=np.int64),
              "out/w": np.asarray([wmap[i] for i in sorted(wmap)], dtype=np.float64),
              "out/w_clip": np.asarray([wclip[i] for i in sorted(wclip)], dtype=np.float64)}
    for bi, b in enumerate(batches):
        for k in KEYS + ("batch", "ptr", "train_idx"):
            arrays[f"in/b{bi}/{k}"] = getattr(b, k).numpy()
    for k, v in model.state_dict().items():
        arrays[f"m/{k}"] = v.numpy()
    arrays["meta/knn"] = np.asarray([KNN[k] for k in ("k", "eps", "alpha", "beta")])
    arrays["meta/clip"] = np.asarray([KNN_CLIP["clip_min"], KNN_CLIP["clip_max"]])
    np.savez_compressed(os.path.join(HERE, "knn.npz"), **arrays)
    print("wrote knn.npz:", len(wmap), "weights, range", min(wmap.values()), max(wmap.values()),
          "clipped range", min(wclip.values()), max(wclip.values()))


if __name__ == "__main__":
    main()
