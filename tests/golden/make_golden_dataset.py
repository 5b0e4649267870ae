"""Golden vectors for the dataset transform from the reference's own code
(build container only).

The reference's ``PtGraphDataset`` (``scripts/train.py:49-216``) and ``_setup`` (``:1300-1447``: group
splits and the train-only feature statistics ``:1324-1380``) run unchanged, through the build's PyG
shim (``oracle/torch_geometric``), over a directory of ``.pt`` graphs this script writes in the
on-disk layout of ``fetch.to_pyg_data`` (``scripts/fetch.py:614-651``: ``global_x [1, 59]``,
``sg_one_hot [1, 230]``).  The directory holds ragged graphs with the production feature widths
(node 206 = 6 scalars + 200 mat2vec, edge 36, angle 11), three of them invalid (NaN in ``x``, +inf in
``lg_edge_attr``, NaN in ``y``) and one without a target — the reference drops all four.

Recorded per mode: the kept graphs, and ``dataset[i].x`` / ``dataset[i].global_x`` for every index:
  * ``setup``    — default dataset, statistics computed by the reference's ``_setup`` (also recorded,
                   with its ``train_idx``), so both the statistics and the transform are pinned;
  * ``shipped``  — default dataset, the statistics of the shipped ensemble
                   (``artifacts/ensemble/scaler_state.pt``, loaded with ``weights_only=True``);
  * ``no_m2v``   — ``use_mat2vec=False`` (scalar block only), shipped scalar/global statistics;
  * ``force100`` — ``force_node_dim=100`` (truncate), shipped statistics cut to 94 mat2vec columns;
  * ``force220`` — ``force_node_dim=220`` (zero pad), shipped statistics + 14 extra columns.

Output: ``tests/golden/dataset.npz`` (allow_pickle=False).  Run: python tests/golden/make_golden_dataset.py
"""
from __future__ import annotations

import os
import sys
import tempfile
from types import SimpleNamespace

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REFERENCE = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))  # shim torch_geometric
sys.path.insert(0, REFERENCE)

import scripts.train as ref  # noqa: E402  (the reference, through the shim)
from torch_geometric.data import Data as ShimData  # noqa: E402

NUM = 24
INVALID = {5: "x_nan", 11: "lg_inf", 17: "y_nan"}
NO_TARGET = 20


def _graph(g: int, rng: np.random.Generator):
    n = int(rng.integers(3, 9))
    e = int(rng.integers(n, 3 * n + 1))
    t = int(rng.integers(e, 3 * e + 1))
    x = np.concatenate([rng.normal(5.0, 3.0, (n, 6)), rng.normal(0.1, 0.3, (n, 200))], 1).astype(np.float32)
    d = dict(
        x=x,
        edge_index=rng.integers(0, n, (2, e)).astype(np.int64),
        edge_attr=rng.normal(0, 1, (e, 36)).astype(np.float32),
        lg_edge_index=rng.integers(0, e, (2, t)).astype(np.int64),
        lg_edge_attr=rng.normal(0, 1, (t, 11)).astype(np.float32),
        global_x=rng.normal(2.0, 4.0, (1, 59)).astype(np.float32),
        sg_one_hot=np.eye(230, dtype=np.float32)[int(rng.integers(0, 230))][None, :],
        y=rng.uniform(1.0, 300.0, (2,)).astype(np.float32),
    )
    if INVALID.get(g) == "x_nan":
        d["x"][1, 3] = np.nan
    if INVALID.get(g) == "lg_inf":
        d["lg_edge_attr"][0, 2] = np.inf
    if INVALID.get(g) == "y_nan":
        d["y"][1] = np.nan
    return d


def _items(ds):
    xs = [ds[i].x.numpy() for i in range(len(ds))]
    gs = [ds[i].global_x.numpy() for i in range(len(ds))]
    return np.concatenate(xs, 0), np.stack([g.reshape(-1) for g in gs], 0)


def main():
    rng = np.random.default_rng(2024)
    graphs = [_graph(g, rng) for g in range(NUM)]
    out = {}
    for k in ("x", "edge_attr", "lg_edge_attr", "global_x", "sg_one_hot", "y"):
        out[f"raw/{k}"] = np.concatenate([d[k].reshape(-1, d[k].shape[-1]) if k != "y" else d[k][None]
                                          for d in graphs], 0)
    out["raw/edge_index"] = np.concatenate([d["edge_index"] for d in graphs], 1)
    out["raw/lg_edge_index"] = np.concatenate([d["lg_edge_index"] for d in graphs], 1)
    out["raw/n"] = np.asarray([d["x"].shape[0] for d in graphs])
    out["raw/e"] = np.asarray([d["edge_index"].shape[1] for d in graphs])
    out["raw/t"] = np.asarray([d["lg_edge_index"].shape[1] for d in graphs])
    out["raw/has_y"] = np.asarray([g != NO_TARGET for g in range(NUM)])
    shipped = torch.load(os.path.join(REFERENCE, "artifacts/ensemble/scaler_state.pt"), weights_only=True)
    with tempfile.TemporaryDirectory() as tmp:
        for g, d in enumerate(graphs):
            data = ShimData(**{k: torch.from_numpy(v.copy()) for k, v in d.items() if k != "y"})
            data.y = None if g == NO_TARGET else torch.from_numpy(d["y"].copy())
            data.material_id = f"mp-{g:03d}"
            torch.save(data, os.path.join(tmp, f"g{g:03d}.pt"))
        args = SimpleNamespace(data_dir=tmp, seed=42, val_frac=0.1, calib_frac=0.05, test_frac=0.1, ensemble_size=5,
                               batch_size=4, num_workers=0, freq_bins=6, freq_gamma=0.0, relative_eps=1e-6)
        dataset, _, _, _, _, scaler_state, train_idx, _, _ = ref._setup(args)
        kept = [int(os.path.basename(str(p))[1:4]) for p in dataset.files]
        out["setup/kept"] = np.asarray(kept)
        out["setup/train_idx"] = np.asarray(train_idx)
        for k in ("scalar_mean", "scalar_std", "embed_mean", "embed_std", "global_mean", "global_std"):
            out[f"setup/stats/{k}"] = scaler_state[k].numpy()
        out["setup/x"], out["setup/global_x"] = _items(dataset)

        sh = {k: shipped[k] for k in ("scalar_mean", "scalar_std", "embed_mean", "embed_std", "global_mean",
                                      "global_std")}
        extra_m, extra_s = torch.full((14,), 0.5), torch.full((14,), 2.0)
        modes = {
            "shipped": (dict(), sh),
            "no_m2v": (dict(use_mat2vec=False), dict(sh, embed_mean=None, embed_std=None)),
            "force100": (dict(force_node_dim=100), dict(sh, embed_mean=sh["embed_mean"][:94],
                                                        embed_std=sh["embed_std"][:94])),
            "force220": (dict(force_node_dim=220), dict(sh, embed_mean=torch.cat([sh["embed_mean"], extra_m]),
                                                        embed_std=torch.cat([sh["embed_std"], extra_s]))),
        }
        for name, (kw, st) in modes.items():
            ds = ref.PtGraphDataset(tmp, **kw)
            ds.set_feature_standardization(st["scalar_mean"], st["scalar_std"], st["embed_mean"], st["embed_std"],
                                           st["global_mean"], st["global_std"])
            out[f"{name}/kept"] = np.asarray([int(os.path.basename(str(p))[1:4]) for p in ds.files])
            out[f"{name}/node_dim"] = np.asarray(ds.node_dim)
            for k, v in st.items():
                if v is not None:
                    out[f"{name}/stats/{k}"] = v.numpy()
            out[f"{name}/x"], out[f"{name}/global_x"] = _items(ds)
    path = os.path.join(HERE, "dataset.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: kept {len(out['setup/kept'])} of {NUM} graphs, train_idx {len(out['setup/train_idx'])}")


if __name__ == "__main__":
    main()
