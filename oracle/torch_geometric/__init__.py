"""ORACLE shim (test infrastructure only, build container only).

A stand-in ``torch_geometric`` package whose arithmetic is :mod:`oracle.pyg_ref` (the build's
restatement of PyG 2.7.0).  It exists so that ``tests/golden/make_golden.py`` can import the
reference's ``scripts/train.py`` (which imports PyG at module top, ``train.py:25-27``) and run the
reference's own model/loss/step code to produce golden vectors.  It is never shipped to or used by
the product path.
"""
from . import data, loader, nn  # noqa: F401
