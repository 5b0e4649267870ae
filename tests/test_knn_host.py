"""KNN density weighting: the oracle's restatement against the weight maps the
reference's own compute_global_knn_weights wrote (sklearn neighbour search), with and without clipping."""
import os

import numpy as np
import torch

from oracle import knn_ref


def test_oracle_knn_weights_match_reference():
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "knn.npz"))
    Z = torch.from_numpy(z["out/Z"])
    Y = torch.cat([torch.from_numpy(z[f"in/b{i}/y"]).view(-1, 2) for i in range(3)]).float()
    idx = torch.cat([torch.from_numpy(z[f"in/b{i}/train_idx"]) for i in range(3)])
    k, eps, alpha, beta = z["meta/knn"]
    lo, hi = z["meta/clip"]
    order = torch.argsort(idx)
    for clip, key in (((None, None), "out/w"), ((float(lo), float(hi)), "out/w_clip")):
        w = knn_ref.knn_weights(Z, Y, int(k), float(eps), float(alpha), float(beta), *clip)
        assert np.allclose(w[order].numpy(), z[key], rtol=1e-5, atol=1e-6), key
