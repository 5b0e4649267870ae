"""Seeded synthetic ALIGNN graphs (SURVEY §8d "Synthetic generator").

* :func:`mp_like_graph` — one "MP-like graph": N=60 atoms, a 12-regular symmetric circulant bond
  graph ``i -> i±1..±6 (mod 60)`` under a seeded atom permutation (E = 720), line graph
  ``(i->j) -> (j->k)`` for k != i (T = 720*11 = 7920; the no-backtrack rule of
  ``scripts/fetch.py:419-447``).  Features ~N(0,1) (standardized features are about N(0,1) after
  ``scripts/train.py:200-216``), one-hot space group, ``y ~ U(1,300)`` (positive for the log
  transform).  Graph ``g`` uses ``torch.Generator().manual_seed(1234 + g)``.
* :func:`si2_smoke_graph` — the shape of the reference's CI fixture (``tests/smoke.py:30-66``):
  Si2 on ``Lattice.cubic(3.5)``, cutoff 5.0 Å, giving N=2, E=58, T=1624 with node/edge/angle dims
  6/8/7.  Periodic neighbours are enumerated with numpy (pymatgen is not available); features are
  seeded random values of the fixture's dims.
"""
from __future__ import annotations

import functools
import itertools
from typing import List, Optional

import numpy as np
import torch

from .data import Batch, Data

GLOBAL_SCALARS = 59
SPACE_GROUPS = 230


def _line_graph(src: np.ndarray, dst: np.ndarray, img: Optional[np.ndarray] = None):
    """Line graph edges (b1 -> b2) for bonds b1=(i->j), b2=(j->k), skipping the exact reverse bond
    (k == i with the reversed image), in the iteration order of fetch.py:419-447."""
    n_atoms = int(max(src.max(), dst.max())) + 1
    out_bonds: List[List[int]] = [[] for _ in range(n_atoms)]
    for b, a in enumerate(src.tolist()):
        out_bonds[a].append(b)
    s_list, d_list = [], []
    for b1 in range(len(src)):
        i, j = int(src[b1]), int(dst[b1])
        for b2 in out_bonds[j]:
            k = int(dst[b2])
            if k == i:
                if img is None or np.array_equal(img[b2], -img[b1]):
                    continue
            s_list.append(b1)
            d_list.append(b2)
    return np.asarray(s_list, dtype=np.int64), np.asarray(d_list, dtype=np.int64)


@functools.lru_cache(maxsize=8)
def _circulant(n_atoms: int, half_degree: int):
    """Bond list of the circulant graph i -> i±1..±half_degree and its line graph in bond indices.
    An atom permutation relabels atoms only: bond b stays bond b, b1 -> b2 is a line-graph edge iff
    dst[b1] == src[b2] and dst[b2] != src[b1] (a bijection preserves both), and the out-bond lists
    keep their order, so every MP-like graph has this same line graph (computed once)."""
    offs = list(range(1, half_degree + 1)) + [-d for d in range(1, half_degree + 1)]
    base_src = np.repeat(np.arange(n_atoms), len(offs))
    base_dst = (base_src + np.tile(np.asarray(offs), n_atoms)) % n_atoms
    lsrc, ldst = _line_graph(base_src, base_dst)
    for a in (base_src, base_dst, lsrc, ldst):
        a.setflags(write=False)
    return base_src, base_dst, lsrc, ldst


def mp_like_graph(g: int, node_dim: int = 206, edge_dim: int = 36, angle_dim: int = 11,
                  n_atoms: int = 60, half_degree: int = 6, target_dim: int = 2) -> Data:
    gen = torch.Generator().manual_seed(1234 + g)
    perm = torch.randperm(n_atoms, generator=gen).numpy()
    base_src, base_dst, lsrc, ldst = _circulant(n_atoms, half_degree)
    src, dst = perm[base_src], perm[base_dst]
    E, T = len(src), len(lsrc)
    sg = torch.zeros(SPACE_GROUPS, 1)
    sg[int(torch.randint(0, SPACE_GROUPS, (1,), generator=gen)), 0] = 1.0
    return Data(
        x=torch.randn(n_atoms, node_dim, generator=gen),
        edge_index=torch.from_numpy(np.stack([src, dst])).long(),
        edge_attr=torch.randn(E, edge_dim, generator=gen),
        lg_edge_index=torch.from_numpy(np.stack([lsrc, ldst])).long(),
        lg_edge_attr=torch.randn(T, angle_dim, generator=gen),
        global_x=torch.randn(GLOBAL_SCALARS, 1, generator=gen),
        sg_one_hot=sg,
        y=torch.rand(target_dim, generator=gen) * 299.0 + 1.0,
    )


def variable_mp_like_graph(g: int, min_atoms: int = 8, max_atoms: int = 60, **kw) -> Data:
    """An MP-like graph of seeded size: n_atoms uniform in [min_atoms, max_atoms], neighbour shells
    half_degree uniform in [2, min(6, (n_atoms - 1) // 2)] (E = 2 half_degree n_atoms bonds,
    T = E (2 half_degree - 1) triplets) — real crystals' spread of sizes for the variable-size loop."""
    r = np.random.default_rng(777 + g)
    n = int(r.integers(min_atoms, max_atoms + 1))
    hd = int(r.integers(2, min(6, (n - 1) // 2) + 1))
    return mp_like_graph(g, n_atoms=n, half_degree=hd, **kw)


def si2_smoke_graph(g: int, cutoff: float = 5.0, a: float = 3.5, node_dim: int = 6, edge_dim: int = 8,
                    angle_dim: int = 7, target_dim: int = 2) -> Data:
    frac = np.array([[0.0, 0.0, 0.0], [0.25, 0.25, 0.25]])
    cart = frac * a
    src, dst, imgs = [], [], []
    rng = range(-3, 4)
    for i in range(2):
        for im in itertools.product(rng, rng, rng):
            for j in range(2):
                d = cart[j] + a * np.asarray(im) - cart[i]
                r = float(np.linalg.norm(d))
                if 1e-8 < r <= cutoff:
                    src.append(i)
                    dst.append(j)
                    imgs.append(im)
    src_a, dst_a, img_a = np.asarray(src), np.asarray(dst), np.asarray(imgs)
    lsrc, ldst = _line_graph(src_a, dst_a, img_a)
    gen = torch.Generator().manual_seed(4321 + g)
    sg = torch.zeros(SPACE_GROUPS, 1)
    sg[227 - 1, 0] = 1.0  # Fd-3m
    return Data(
        x=torch.randn(2, node_dim, generator=gen),
        edge_index=torch.from_numpy(np.stack([src_a, dst_a])).long(),
        edge_attr=torch.randn(len(src_a), edge_dim, generator=gen),
        lg_edge_index=torch.from_numpy(np.stack([lsrc, ldst])).long(),
        lg_edge_attr=torch.randn(len(lsrc), angle_dim, generator=gen),
        global_x=torch.randn(GLOBAL_SCALARS, 1, generator=gen),
        sg_one_hot=sg,
        y=torch.tensor([100.0 + g, 60.0 + g])[:target_dim],
    )


def mp_like_batch(num_graphs: int, first: int = 0, lg_offset: str = "num_nodes", **kw) -> Batch:
    return Batch.from_data_list([mp_like_graph(first + g, **kw) for g in range(num_graphs)],
                                lg_offset=lg_offset)


def ensemble_member_batch(num_graphs: int, member: int, fold: int, lg_offset: str = "num_nodes") -> Batch:
    """Member ``member``'s synthetic training batch: graphs of its fold (train.py:2054) — a slice
    disjoint from every other member's and from the headline batches."""
    return mp_like_batch(num_graphs, first=100000 * (1 + int(fold)) + 1000 * int(member), lg_offset=lg_offset)


# LogTransformer statistics of the shipped ensemble (artifacts/ensemble/scaler_state.pt)
TARGET_LOG_MEANS = (4.3228, 3.5567)
TARGET_LOG_STDS = (0.9051, 0.9405)
