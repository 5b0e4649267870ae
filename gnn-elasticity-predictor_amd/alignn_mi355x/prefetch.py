"""Background batch preparation for the training loop over an HBM-resident dataset.

The reference's loop (train.py:639-711) draws each batch from a PyG ``DataLoader`` whose worker
processes collate on the host while the step runs.  Here the dataset is resident in HBM
(``store.GraphStore``) and a batch is collated and prepared on the device (``GraphStore.collate`` +
``engine.prepare_batch``: CSR lists, line-graph compaction, schedules), but issuing that work still
costs host time — about as much as the step's own host side (plan re-binding + replay).  A
``BatchPrefetcher`` issues it from a host thread on its own loader stream, ``depth`` batches ahead:
the step's host work (whose native calls — plan replay, the re-binding copy — run without the
interpreter lock) and the next batches' preparation overlap instead of adding up.

Ordering and memory are those of ``prepare_batch``: each batch carries the event its preparation
recorded on the loader stream; the consuming step waits for it and marks the batch's buffers as used
by its own stream (``engine.adopt``), so the caching allocator never hands them back to the loader
while the step may still read them.  Index draws happen in the thread in a fixed order, so the batch
sequence is the one a synchronous loop with the same index source produces.
"""
from __future__ import annotations

import queue
import threading
from typing import Callable, Optional

import numpy as np
import torch

_STOP = object()


class BatchPrefetcher:
    """Prepared batches of ``store``, in the order ``next_indices()`` draws them.

    next_indices: callable returning the next batch's graph indices (numpy int array), or None to end.
    depth: batches prepared ahead (each holds its collated fields and cache in HBM).
    lg_offset / capacity: as ``GraphStore.collate``.  priority: the loader stream's HIP priority.
    """

    def __init__(self, store, next_indices: Callable[[], Optional[np.ndarray]], depth: int = 2,
                 lg_offset: str = "num_nodes", capacity=None, priority: int = 0, validate: bool = True):
        if depth < 1:
            raise ValueError("depth must be >= 1")
        self.store = store
        self.device = next(iter(store.arrays.values())).device
        if self.device.type != "cuda":
            raise ValueError("BatchPrefetcher needs a store resident on the HIP device")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self._next = next_indices
        self._lg_offset, self._capacity, self._validate = lg_offset, capacity, validate
        self._q: "queue.Queue" = queue.Queue(maxsize=depth)
        self._stop = threading.Event()
        self._stream = torch.cuda.Stream(device=self.device, priority=priority)
        self.produced = 0
        self._thread = threading.Thread(target=self._run, name="alignn-prefetch", daemon=True)
        self._thread.start()

    def _put(self, item) -> bool:
        while not self._stop.is_set():
            try:
                self._q.put(item, timeout=0.1)
                return True
            except queue.Full:
                continue
        return False

    def _run(self) -> None:
        from .engine import prepare_batch
        try:
            torch.cuda.set_device(self.device)
            while not self._stop.is_set():
                idx = self._next()
                if idx is None:
                    break
                with torch.cuda.stream(self._stream):
                    b = self.store.collate(idx, lg_offset=self._lg_offset, capacity=self._capacity)
                prepare_batch(b, self._stream, validate=self._validate)
                self.produced += 1
                if not self._put(b):
                    return
        except BaseException as e:  # noqa: BLE001 - re-raised in the consumer
            self._put(e)
            return
        self._put(_STOP)

    def get(self):
        """The next prepared batch (blocks until it is ready on the host side; its device work may
        still be in flight — the step waits for its event).  Raises StopIteration at the end and
        re-raises an error of the loader thread."""
        item = self._q.get()
        if item is _STOP:
            self._q.put(_STOP)
            raise StopIteration
        if isinstance(item, BaseException):
            self._q.put(item)
            raise item
        return item

    def __iter__(self):
        return self

    def __next__(self):
        return self.get()

    def close(self) -> None:
        """Stops the thread (batches already prepared are dropped)."""
        self._stop.set()
        try:
            while True:
                self._q.get_nowait()
        except queue.Empty:
            pass
        self._thread.join(timeout=30)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False
