"""KNN density weighting on the engine vs the weight maps written by the reference's
compute_global_knn_weights (tests/golden/make_golden_knn.py).  Sorts after the core suites."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
KEYS = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y", "batch",
        "ptr", "train_idx")


def test_knn_weights_match_reference():
    import alignn_mi355x as A
    from alignn_mi355x.knn import compute_global_knn_weights, embed_collect
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "knn.npz"))
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 64, 2, 4, 0.15), 2)
    model.load_state_dict({k[2:]: torch.from_numpy(np.array(z[k])) for k in z.files if k.startswith("m/")})
    model.to(DEV)
    batches = []
    for bi in range(3):
        b = A.Batch()
        for k in KEYS:
            setattr(b, k, torch.from_numpy(np.array(z[f"in/b{bi}/{k}"])))
        b.num_graphs = int(b.ptr.numel() - 1)
        batches.append(b.to(DEV))
    Z, _, _ = embed_collect(model, batches)
    assert float((Z.cpu() - torch.from_numpy(z["out/Z"])).abs().max()) < 1e-4 * float(np.abs(z["out/Z"]).max())
    k, eps, alpha, beta = (float(v) for v in z["meta/knn"])
    lo, hi = (float(v) for v in z["meta/clip"])
    for clip, key in (((None, None), "out/w"), ((lo, hi), "out/w_clip")):
        wm = compute_global_knn_weights(model, batches, k=int(k), eps=eps, alpha=alpha, beta=beta,
                                        clip_min=clip[0], clip_max=clip[1])
        got = np.asarray([wm[int(i)] for i in z["out/idx"]])
        assert np.allclose(got, z[key], rtol=1e-4, atol=1e-5), key
