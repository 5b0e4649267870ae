"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement of the reference's deep-ensemble inference math.  Pinned by
``tests/golden/ensemble.npz``, which the reference's own functions wrote
(``tests/golden/make_golden_ensemble.py``); ``predict_moments`` restates predict.py, which imports
pymatgen and cannot be imported here — its moment mix is the pinned one, the log-normal conversion
is a closed form checked by hand-computed values (parity partially unpinned for that step).
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Sequence, Tuple

import numpy as np
import torch

Z_SCORE_90 = 1.6448536269514722  # predict.py:63


def mixture(means: Sequence[torch.Tensor], logvars: Sequence[torch.Tensor], floor: float):
    """ensemble_collect's moment mix (train.py:875-894): returns mean_z, var_z."""
    mu = torch.stack(list(means), 0)
    var = torch.stack([torch.exp(torch.clamp(lv, min=floor)) for lv in logvars], 0)
    mean_z = mu.mean(0)
    var_z = var.mean(0) + mu.pow(2).mean(0) - mean_z.pow(2)
    return mean_z, var_z


def std_from_var(var_z: torch.Tensor) -> torch.Tensor:
    return torch.sqrt(torch.clamp(var_z, min=1e-12))  # train.py:902, predict.py:614


def predict_moments(mean_z, std_z, log_means, log_stds) -> Dict[str, torch.Tensor]:
    """predict.ensemble_predict (predict.py:616-640): target-scale mean, log-normal std, 90% CI."""
    m = torch.as_tensor(log_means, dtype=mean_z.dtype)
    s = torch.as_tensor(log_stds, dtype=mean_z.dtype)
    log_mean = mean_z * s + m
    mean_orig = torch.exp(log_mean)
    log_std = std_z * s
    var_lin = (torch.exp(log_std.pow(2)) - 1.0) * torch.exp(2 * log_mean + log_std.pow(2))
    std_lin = torch.sqrt(torch.clamp(var_lin, min=0.0))
    return {"mean_orig": mean_orig, "std_lin": std_lin,
            "lo90": torch.clamp(mean_orig - Z_SCORE_90 * std_lin, min=0.0), "hi90": mean_orig + Z_SCORE_90 * std_lin}


def fit_affine(pred_z: torch.Tensor, target_z: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """_fit_affine_debias (train.py:1013-1026): per-target least squares target ~ a*pred + b."""
    p = pred_z.double().numpy()
    t = target_z.double().numpy()
    a, b = [], []
    for k in range(p.shape[1]):
        X = np.stack([p[:, k], np.ones_like(p[:, k])], 1)
        sol = np.linalg.lstsq(X, t[:, k], rcond=None)[0]
        a.append(sol[0])
        b.append(sol[1])
    return torch.tensor(a), torch.tensor(b)


def conformal_q(mean_z, std_z, targets, log_means, log_stds, alpha: float, method: str):
    """conformal_calibration (train.py:1029-1051)."""
    tz = (torch.log(torch.clamp(targets, min=1e-12)) - torch.as_tensor(log_means, dtype=targets.dtype)) / \
        torch.as_tensor(log_stds, dtype=targets.dtype)
    if method == "scaled" and std_z is not None:
        s = (tz - mean_z).abs() / torch.clamp(std_z, min=1e-12)
    else:
        s = (tz - mean_z).abs()
        method = "absolute"
    n = s.size(0)
    q_level = min(max(math.ceil((n + 1) * (1 - alpha)) / n, 0.0), 1.0)
    return torch.quantile(s, q_level, dim=0), method
