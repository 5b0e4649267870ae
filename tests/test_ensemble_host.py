"""Ensemble inference, host side: the oracle's restatement against the golden vectors
the reference's own ensemble_collect / conformal / affine functions wrote, and the product's
calibration functions (which run on the host, like the reference's) against the same vectors."""
import math

import numpy as np
import pytest
import torch

from _golden_util import rel_err
from oracle import ensemble_ref, model_ref
from oracle.pyg_ref import RefData

KEYS = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y", "batch",
        "ptr")


@pytest.fixture(scope="module")
def ens():
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "ensemble.npz"))
    return {k: z[k] for k in z.files}


def _ref_batches(g, dtype=torch.float64):
    out = []
    for bi in range(2):
        kw = {}
        for k in KEYS:
            v = torch.from_numpy(np.array(g[f"in/b{bi}/{k}"]))
            kw[k] = v.to(dtype) if v.is_floating_point() else v
        b = RefData(**kw)
        b.num_graphs = int(kw["ptr"].numel() - 1)
        out.append(b)
    return out


def _members(g, dtype=torch.float64):
    return [{k[3:]: torch.from_numpy(np.array(v)).to(dtype) for k, v in g.items() if k.startswith(f"m{j}/")}
            for j in range(3)]


def test_oracle_mixture_matches_reference_ensemble_collect(ens):
    """Members' forwards (oracle, fp64) + the oracle moment mix == the reference's ensemble_collect."""
    floor = float(ens["meta/min_logvar_floor"])
    heads = int(ens["meta/dims"][6])
    means, stds = [], []
    for b in _ref_batches(ens):
        mus, lvs = [], []
        for st in _members(ens):
            mu, lv = model_ref.hetero_forward(st, b, heads)
            mus.append(mu)
            lvs.append(lv)
        m, v = ensemble_ref.mixture(mus, lvs, floor)
        means.append(m)
        stds.append(ensemble_ref.std_from_var(v))
    assert rel_err(torch.cat(means), ens["out/mean_z"]) < 1e-5
    assert rel_err(torch.cat(stds), ens["out/std_z"]) < 1e-5


def test_affine_and_conformal_match_reference(ens):
    from alignn_mi355x import ensemble as E
    lm, ls = ens["meta/target_log_means"], ens["meta/target_log_stds"]
    mean_z = torch.from_numpy(ens["out/mean_z"])
    std_z = torch.from_numpy(ens["out/std_z"])
    targets = torch.from_numpy(ens["out/targets"])
    tz = (torch.log(targets) - torch.from_numpy(lm).float()) / torch.from_numpy(ls).float()
    a, b = E.fit_affine_debias(mean_z, tz)
    assert rel_err(a, ens["out/affine_a"]) < 1e-5 and rel_err(b, ens["out/affine_b"]) < 1e-5
    oa, ob = ensemble_ref.fit_affine(mean_z, tz)
    assert rel_err(oa, ens["out/affine_a"]) < 1e-5 and rel_err(ob, ens["out/affine_b"]) < 1e-5
    for method in ("scaled", "absolute"):
        conf = E.conformal_calibration(mean_z, std_z, targets, 0.1, method, lm.tolist(), ls.tolist())
        assert conf["method"] == method
        assert rel_err(conf["q"], ens[f"out/conformal_{method}/q"]) < 1e-6
        q_o, _ = ensemble_ref.conformal_q(mean_z, std_z, targets, lm.tolist(), ls.tolist(), 0.1, method)
        assert rel_err(q_o, ens[f"out/conformal_{method}/q"]) < 1e-6
        for name, t in zip(("mean", "lower", "upper"),
                           E.apply_conformal_intervals(mean_z, std_z, conf, lm.tolist(), ls.tolist())):
            assert rel_err(t, ens[f"out/conformal_{method}/{name}"]) < 1e-6, (method, name)


def test_predict_moments_known_answer():
    """predict.py:616-640 by hand: one target, log-space mean 0.5 / std 0.2 after de-standardizing."""
    mean_z = torch.tensor([[0.5]], dtype=torch.float64)
    std_z = torch.tensor([[0.1]], dtype=torch.float64)
    r = ensemble_ref.predict_moments(mean_z, std_z, [0.0], [2.0])
    lm, lsd = 1.0, 0.2
    mo = math.exp(lm)
    sl = math.sqrt((math.exp(lsd ** 2) - 1) * math.exp(2 * lm + lsd ** 2))
    assert abs(float(r["mean_orig"]) - mo) < 1e-12
    assert abs(float(r["std_lin"]) - sl) < 1e-12
    assert abs(float(r["lo90"]) - max(mo - ensemble_ref.Z_SCORE_90 * sl, 0.0)) < 1e-12
    assert abs(float(r["hi90"]) - (mo + ensemble_ref.Z_SCORE_90 * sl)) < 1e-12
