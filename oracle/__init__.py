"""ORACLE — test infrastructure only.

A PyTorch-CPU restatement of the reference's hot path (conorjmoran/gnn-elasticity-predictor,
``scripts/train.py``) and of the third-party PyG 2.7.0 pieces it calls (``TransformerConv``,
``utils.softmax``, ``global_mean_pool``, ``Batch.from_data_list``).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
package, and only as the checker / the CPU baseline.  The product path
(``gnn-elasticity-predictor_amd/alignn_mi355x``) never imports it and has no CPU fallback.

Parity status
-------------
* Model composition, block structure, readout, loss, clip and AdamW: pinned against golden
  vectors produced by the reference's own ``scripts/train.py`` classes (imported in the build
  container through :mod:`oracle.torch_geometric`, see ``tests/golden/make_golden.py``).
* ``TransformerConv`` / segment softmax / mean pool / collate arithmetic: PyG 2.7.0
  (``requirements.txt:9``) is absent from the container, so these are restated from PyG's
  published algorithm and pinned by hand-computed known-answer tests
  (``tests/test_oracle_kat.py``) — *parity with real PyG is unpinned* beyond that.
"""
