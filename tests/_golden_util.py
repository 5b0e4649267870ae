"""Helpers to turn a golden .npz into (state dict, batch) for oracle / engine tests."""
import numpy as np
import torch

INPUT_KEYS = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x",
              "sg_one_hot", "y", "batch", "ptr")


def state_from(g, prefix="p/", dtype=torch.float32):
    return {k[len(prefix):]: torch.from_numpy(np.array(v)).to(dtype) for k, v in g.items()
            if k.startswith(prefix)}


def batch_from(g, cls, dtype=torch.float32):
    b = cls()
    for k in INPUT_KEYS:
        v = torch.from_numpy(np.array(g[f"in/{k}"]))
        if v.is_floating_point():
            v = v.to(dtype)
        setattr(b, k, v)
    b.num_graphs = int(g["meta/num_graphs"])
    return b


def meta(g):
    return {k[5:]: g[k].item() if g[k].ndim == 0 else g[k] for k in g if k.startswith("meta/")}


def rel_err(a, b, floor=1e-30):
    """max|a-b| / max(max|b|, floor).  ``floor`` guards tensors that are 0 in exact arithmetic
    (e.g. lin_key.bias grads: a per-segment constant shift cancels in the softmax)."""
    a = torch.as_tensor(a, dtype=torch.float64).detach()
    b = torch.as_tensor(b, dtype=torch.float64).detach()
    if a.numel() == 0:
        return 0.0
    return float((a - b).abs().max() / b.abs().max().clamp(min=floor))


def grad_scale(g, tag):
    """Largest |grad| over all parameters of a golden case (used as the floor for rel_err)."""
    import numpy as np
    return max(float(np.abs(v).max()) for k, v in g.items() if k.startswith(f"{tag}/grad/"))


def norm_err(a, b, floor=0.0):
    """||a-b||_F / max(||b||_F, floor): the gradient criterion.  A max-abs criterion is ill-posed for
    gradients behind ReLUs: an activation within fp32 rounding of 0 can take the other side of the
    kink than in the fp64 reference, which moves single gradient entries by O(1) relative."""
    a = torch.as_tensor(a, dtype=torch.float64).detach().cpu()
    b = torch.as_tensor(b, dtype=torch.float64).detach().cpu()
    if a.numel() == 0:
        return 0.0
    return float((a - b).norm() / max(float(b.norm()), floor, 1e-30))


def grad_norm_scale(grads):
    return max(float(torch.as_tensor(v, dtype=torch.float64).norm()) for v in grads)


def dataset_graphs(z):
    """The raw on-disk graphs of tests/golden/dataset.npz as dicts of CPU tensors (fetch.to_pyg_data
    layout: global_x [1, 59], sg_one_hot [1, 230]; y None for the graph without a target)."""
    n, e, t = (np.asarray(z[f"raw/{k}"]) for k in ("n", "e", "t"))
    cut = lambda a, c, ax=0: np.split(np.asarray(a), np.cumsum(c)[:-1], axis=ax)  # noqa: E731
    G = len(n)
    parts = {
        "x": cut(z["raw/x"], n), "edge_attr": cut(z["raw/edge_attr"], e), "lg_edge_attr": cut(z["raw/lg_edge_attr"], t),
        "edge_index": cut(z["raw/edge_index"], e, 1), "lg_edge_index": cut(z["raw/lg_edge_index"], t, 1),
        "global_x": [r[None] for r in np.asarray(z["raw/global_x"])],
        "sg_one_hot": [r[None] for r in np.asarray(z["raw/sg_one_hot"])], "y": list(np.asarray(z["raw/y"])),
    }
    out = []
    for g in range(G):
        d = {k: torch.from_numpy(np.ascontiguousarray(v[g])) for k, v in parts.items()}
        if not bool(z["raw/has_y"][g]):
            d["y"] = None
        out.append(d)
    return out


DATASET_MODES = {"setup": {}, "shipped": {}, "no_m2v": {"use_mat2vec": False}, "force100": {"force_node_dim": 100},
                 "force220": {"force_node_dim": 220}}


def dataset_stats(z, mode):
    keys = ("scalar_mean", "scalar_std", "embed_mean", "embed_std", "global_mean", "global_std")
    return {k: (torch.from_numpy(np.asarray(z[f"{mode}/stats/{k}"])) if f"{mode}/stats/{k}" in z else None)
            for k in keys}
