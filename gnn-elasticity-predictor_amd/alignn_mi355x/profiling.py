"""Per-launch HIP-event probes for the roofline report (bench.py).

``ops`` calls :func:`record` around every launch when probing is enabled.  Events are recorded on
the current stream (the one the kernel is launched on), so elapsed times are device times of that
launch.  Probing is off by default and costs nothing then.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Callable, Dict, List, Optional, Tuple

import torch

_enabled = False
_only: Optional[str] = None
_events: Dict[str, List[Tuple[torch.cuda.Event, torch.cuda.Event, float, float]]] = defaultdict(list)


def enable(only: Optional[str] = None) -> None:
    global _enabled, _only
    _enabled, _only = True, only
    _events.clear()


def clear() -> None:
    """Drop recorded events (keeps the enabled state)."""
    _events.clear()


def disable() -> None:
    global _enabled
    _enabled = False


def active(key: str) -> bool:
    return _enabled and (_only is None or _only == key)


def launch(key: str, flops: float, nbytes: float, fn: Callable[[], None]) -> None:
    """Run ``fn`` (one kernel launch sequence) with start/end events if ``key`` is probed."""
    if not active(key):
        fn()
        return
    # inside HIP-graph capture the events become event-record nodes of the graph (external), so
    # after a replay they hold that replay's device times of this launch
    ext = torch.cuda.is_current_stream_capturing()
    s = torch.cuda.Event(enable_timing=True, external=ext)
    e = torch.cuda.Event(enable_timing=True, external=ext)
    s.record()
    fn()
    e.record()
    _events[key].append((s, e, flops, nbytes))


def summary() -> Dict[str, dict]:
    """key -> {count, total_ms, avg_ms, flops_per_launch, bytes_per_launch}; call after a sync."""
    out = {}
    for k, evs in _events.items():
        ms = [s.elapsed_time(e) for s, e, _, _ in evs]
        out[k] = {
            "count": len(ms),
            "total_ms": sum(ms),
            "avg_ms": sum(ms) / len(ms),
            "flops_per_launch": sum(f for _, _, f, _ in evs) / len(evs),
            "bytes_per_launch": sum(b for _, _, _, b in evs) / len(evs),
        }
    return out
