"""Per-launch HIP-event probes for the roofline report (bench.py).

``ops`` calls :func:`record` around every launch when probing is enabled.  Events are recorded on
the current stream (the one the kernel is launched on), so elapsed times are device times of that
launch.  While a launch plan is being recorded (trainer.capture, mode "plan") the probe becomes a
pair of plan timestamps instead: every replay re-records them, so after a replay they hold that
replay's device time of the launch.  Probing is off by default and costs nothing then.
"""
from __future__ import annotations

from collections import defaultdict
from typing import Callable, Dict, List, Optional, Tuple

import torch

_enabled = False
_only: Optional[str] = None
_events: Dict[str, List[Tuple[torch.cuda.Event, torch.cuda.Event, float, float]]] = defaultdict(list)
_plan_recording = False
_plan_pending: List[Tuple[str, int, int, float, float]] = []
_plan_probes: Dict[str, List[Tuple[int, int, int, float, float]]] = defaultdict(list)


def enable(only: Optional[str] = None) -> None:
    global _enabled, _only
    _enabled, _only = True, only
    clear()


def clear() -> None:
    """Drop recorded events and plan probes (keeps the enabled state)."""
    _events.clear()
    _plan_pending.clear()
    _plan_probes.clear()


def plan_recording(on: bool) -> None:
    """Set by the trainer around the recording of a launch plan."""
    global _plan_recording
    _plan_recording = on
    if on:
        _plan_pending.clear()


def bind_plan(plan: int) -> None:
    """Attach the probes noted during the recording that produced ``plan``."""
    for key, i0, i1, f, b in _plan_pending:
        _plan_probes[key].append((plan, i0, i1, f, b))
    _plan_pending.clear()


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
    if _plan_recording:
        from . import _lib
        stream = torch.cuda.current_stream().cuda_stream
        i0 = _lib.lib().alignn_plan_note_timestamp(stream)
        fn()
        i1 = _lib.lib().alignn_plan_note_timestamp(stream)
        if i0 >= 0 and i1 >= 0:
            _plan_pending.append((key, i0, i1, flops, nbytes))
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
    timed = {k: [(s.elapsed_time(e), f, b) for s, e, f, b in evs] for k, evs in _events.items()}
    if _plan_probes:
        import ctypes

        from . import _lib
        from ._lib import check
        for k, probes in _plan_probes.items():
            for plan, i0, i1, f, b in probes:
                ms = ctypes.c_float()
                check(_lib.lib().alignn_plan_elapsed_ms(plan, i0, i1, ctypes.byref(ms)), "alignn_plan_elapsed_ms")
                timed.setdefault(k, []).append((ms.value, f, b))
    for k, evs in timed.items():
        ms = [t for t, _, _ in evs]
        out[k] = {
            "count": len(ms),
            "total_ms": sum(ms),
            "avg_ms": sum(ms) / len(ms),
            "flops_per_launch": sum(f for _, f, _ in evs) / len(evs),
            "bytes_per_launch": sum(b for _, _, b in evs) / len(evs),
        }
    return out
