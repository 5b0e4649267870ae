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
