"""Ensemble inference on the engine against the golden vectors written by the
reference's ensemble_collect / ensemble_collect_embeddings (tests/golden/make_golden_ensemble.py),
and predict.ensemble_predict's conversions against the oracle.  Sorts after the core suites."""
import os

import numpy as np
import pytest
import torch

from _golden_util import rel_err
from oracle import ensemble_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-4
KEYS = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y", "batch",
        "ptr")


@pytest.fixture(scope="module")
def ens():
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "ensemble.npz"))
    return {k: z[k] for k in z.files}


def _setup(g, concurrent=True):
    import alignn_mi355x as A
    from alignn_mi355x.ensemble import EnsemblePredictor
    node, edge, angle, glob, hidden, layers, heads = (int(v) for v in g["meta/dims"])
    models = []
    for j in range(3):
        m = A.HeteroAlignnRegressor(A.AlignnRegressor(node, edge, angle, glob, 2, hidden, layers, heads, 0.15), 2)
        m.load_state_dict({k[3:]: torch.from_numpy(np.array(v)) for k, v in g.items() if k.startswith(f"m{j}/")})
        models.append(m.to(DEV).eval())
    batches = []
    for bi in range(2):
        b = A.Batch()
        for k in KEYS:
            setattr(b, k, torch.from_numpy(np.array(g[f"in/b{bi}/{k}"])))
        b.num_graphs = int(b.ptr.numel() - 1)
        batches.append(b.to(DEV))
    ep = EnsemblePredictor(models, float(g["meta/min_logvar_floor"]), g["meta/target_log_means"].tolist(),
                           g["meta/target_log_stds"].tolist(), concurrent=concurrent)
    return ep, batches


def test_collect_and_embed_match_reference(ens):
    ep, batches = _setup(ens)
    mean_z, targets, std_z = ep.collect(batches)
    assert rel_err(mean_z, ens["out/mean_z"]) < TOL
    assert rel_err(std_z, ens["out/std_z"]) < TOL
    assert torch.equal(targets, torch.from_numpy(ens["out/targets"]))
    assert rel_err(ep.embed(batches), ens["out/embed"]) < TOL


def test_predict_batch_matches_oracle_conversion(ens):
    ep, batches = _setup(ens)
    r = ep.predict_batch(batches[0])
    o = ensemble_ref.predict_moments(r["mean_z"].cpu().double(), r["std_z"].cpu().double(),
                                     ens["meta/target_log_means"], ens["meta/target_log_stds"])
    for k in ("mean_orig", "std_lin", "lo90", "hi90"):
        assert rel_err(r[k].cpu(), o[k]) < 1e-5, k


def test_concurrent_members_equal_sequential_bitwise(ens):
    ep1, b1 = _setup(ens, concurrent=True)
    ep2, b2 = _setup(ens, concurrent=False)
    h1 = ep1.member_outputs(b1[1])
    h2 = ep2.member_outputs(b2[1])
    torch.cuda.synchronize()
    assert torch.equal(h1, h2)


def test_sharded_ensemble_world1_matches_reference(ens):
    """ShardedEnsemble (members over ranks, RCCL gather to rank 0) in a 1-rank group holds all three
    members; its collect/embed are the reference's.  Multi-rank placement and gather order are
    covered by tests/test_dp_gloo.py."""
    import torch.distributed as dist
    from alignn_mi355x.ensemble import ShardedEnsemble
    ep, batches = _setup(ens)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1)
    try:
        se = ShardedEnsemble(ep.models, 3, target_dim=2, hidden=int(ens["meta/dims"][4]),
                             min_logvar_floor=float(ens["meta/min_logvar_floor"]),
                             target_log_means=ens["meta/target_log_means"].tolist(),
                             target_log_stds=ens["meta/target_log_stds"].tolist())
        mean_z, targets, std_z = se.collect(batches)
        emb = se.embed(batches)
        r = se.predict_batch(batches[0])
    finally:
        dist.destroy_process_group()
    assert rel_err(mean_z, ens["out/mean_z"]) < TOL
    assert rel_err(std_z, ens["out/std_z"]) < TOL
    assert torch.equal(targets, torch.from_numpy(ens["out/targets"]))
    assert rel_err(emb, ens["out/embed"]) < TOL
    r0 = ep.predict_batch(batches[0])
    for k in r0:
        assert torch.equal(r[k], r0[k]), k
