"""Tensor-level wrappers over the C ABI (``_lib``).  Torch tensors provide device memory, strides
and the current HIP stream; all arithmetic runs in ``libalignn_hip.so``.  No fallbacks."""
from __future__ import annotations

import ctypes
import math
import threading
from contextlib import contextmanager
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch

from . import _lib, profiling
from ._lib import GemmArgs, check



def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def _require(t: torch.Tensor, name: str, dtype=torch.float32):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device (HIP) tensor; the engine has no CPU path")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")


# ------------------------------------------------------------------------------------------------
# Execution context: scratch workspaces, auxiliary streams and the device step seed of one engine
# ------------------------------------------------------------------------------------------------
_DEDICATED: dict = {}


_WARMUP: dict = {}


def warmup_stream(device) -> torch.cuda.Stream:
    """One stream per device, kept for the process, for the warm-up passes before a capture
    (FusedTrainer.capture, infer.ForwardPlan).  A fresh pooled stream per capture made a new HIP stream
    (and hardware-queue assignment) every time: after a second capture in the process the B = 32 e2e
    loop's loader stream ran ~25 % slower (7,200-7,700 vs 10,000 graphs/s, gpurun_out r6z-r6ac)."""
    key = _dkey(device)
    s = _WARMUP.get(key)
    if s is None:
        s = _WARMUP[key] = torch.cuda.Stream(device=torch.device(key))
    return s


def dedicated_stream(device) -> torch.cuda.Stream:
    """A stream on a hardware queue of its own (alignn_stream_create_dedicated), one per device, kept
    for the process: for a batch-preparation stream beside a replayed step.  With the process's
    pooled queues (GPU_MAX_HW_QUEUES = 4) a loader stream could share a queue with one of the step's
    streams, and its kernels then wait behind the step's in queue order."""
    key = _dkey(device)
    h = _DEDICATED.get(key)
    if h is None:
        hv = ctypes.c_void_p()
        with torch.cuda.device(torch.device(key)):
            check(_lib.lib().alignn_stream_create_dedicated(ctypes.byref(hv)), "alignn_stream_create_dedicated")
        h = _DEDICATED[key] = hv.value
    return torch.cuda.ExternalStream(h, device=torch.device(key))


def _dkey(device) -> str:
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return str(d)


_FREE_STREAMS: dict = {}   # (device, priority) -> library streams no live context holds
# HIP priority of the side / aux streams contexts create from now on (0 normal, -1 high): with the
# caller's step stream also at -1, a loader stream at 0 only takes what the step leaves idle
STREAM_PRIORITY = 0


class ExecContext:
    """What the launches of one engine (model) share: per-purpose scratch buffers, the side / aux
    streams for work off the critical path, and the device step seed its dropout kernels read.

    Buffers are keyed by (purpose, device, dtype, stream role).  In an engine-owned context the role
    is "main" (whatever stream is current: a plan is recorded on a capture stream and replayed on
    another), "side" or "aux" (this context's own streams); in the shared default context it is the
    stream itself.  Kernels on different streams therefore never share one, and a buffer is reused
    only in its stream's order.  A buffer grows on demand while nothing is being recorded; during a
    launch-plan recording (:func:`recording`) growth is refused, because earlier recorded launches
    hold the old buffer's address.  While a recorded plan is alive (:meth:`freeze`) a buffer is never
    replaced either: an eager launch that needs more than a plan's buffer gets a separate one, so
    the plan's addresses stay valid.  The trainer sizes them with uncaptured warm-up steps of the same
    shapes first and owns them for as long as its plans live.

    ``fresh(purpose, ...)`` hands out a distinct buffer per call within one backward pass (reset by
    :meth:`new_pass`): for data written on one stream and read later on another (the gate/LayerNorm
    parameter-gradient partials, reduced on the side stream)."""

    def __init__(self, name: str = "engine", owned: bool = True):
        self.name = name
        self.owned = owned
        self.buf = {}
        self._cursor = {}
        self._side = {}
        self._aux = {}
        self.step_seed: Optional[torch.Tensor] = None
        self._owned_streams = []
        self.frozen = 0       # live plans / graphs holding this context's buffers
        self._eager = {}      # buffers of eager launches that outgrew a frozen buffer
        self._lender = None   # borrow_streams

    def freeze(self) -> None:
        """A recorded plan now holds this context's buffers: none may be replaced while it lives."""
        self.frozen += 1

    def thaw(self) -> None:
        """A plan holding the buffers was released; with none left, eager overflow buffers become
        the regular ones."""
        self.frozen = max(0, self.frozen - 1)
        if self.frozen == 0:
            for k, t in self._eager.items():
                cur = self.buf.get(k)
                if cur is None or cur.numel() < t.numel():
                    self.buf[k] = t
            self._eager.clear()

    def _own_stream(self, device) -> torch.cuda.Stream:
        """A stream created by the library (alignn_stream_create), not taken from torch's pool: pooled
        streams repeat after 32 and could coincide with a capture or caller stream, which this context
        would then mistake for its side / aux stream.  Held by one live context at a time; a released
        one is reused, never destroyed (tensors recorded on it may outlive the context)."""
        key = _dkey(device)
        prio = int(STREAM_PRIORITY)
        free = _FREE_STREAMS.setdefault((key, prio), [])
        if free:
            h = free.pop()
        else:
            hv = ctypes.c_void_p()
            check(_lib.lib().alignn_stream_create(prio, ctypes.byref(hv)), "alignn_stream_create")
            h = hv.value
        self._owned_streams.append(((key, prio), h))
        return torch.cuda.ExternalStream(h, device=torch.device(key))

    def borrow_streams(self, other: "ExecContext") -> None:
        """Take ``other``'s side / aux streams instead of creating this context's own, for an engine
        that never runs at the same time as ``other``'s (bench.py's secondary configurations, measured
        beside the idle headline trainer).  The process then holds no more streams than one engine
        needs: with GPU_MAX_HW_QUEUES = 4, each extra stream shares a hardware queue with one of the
        step's, whose kernels then wait behind each other in queue order (C3 measured 21,640 beside
        the headline trainer's own streams vs 23,515 graphs/s alone; profiles/r05/v16_*)."""
        if self._side or self._aux:
            raise RuntimeError("borrow_streams: this context already has streams of its own")
        self._lender = other

    def side(self, device) -> torch.cuda.Stream:
        """A second stream per device for work off the critical path (weight gradients)."""
        key = _dkey(device)
        if key not in self._side:
            self._side[key] = self._lender.side(device) if self._lender is not None else self._own_stream(device)
        return self._side[key]

    def aux(self, device) -> torch.cuda.Stream:
        """A third stream per device for short branches beside the critical path."""
        key = _dkey(device)
        if key not in self._aux:
            self._aux[key] = self._lender.aux(device) if self._lender is not None else self._own_stream(device)
        return self._aux[key]

    def __del__(self):
        try:
            for kp, h in self._owned_streams:
                _FREE_STREAMS.setdefault(kp, []).append(h)
            self._owned_streams = []
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    def _role(self, device):
        if torch.device(device).type != "cuda":
            return "main"
        cur = torch.cuda.current_stream(device).cuda_stream
        if not self.owned:
            return ("stream", cur)   # shared context: one buffer per stream (loader and main never share)
        key = _dkey(device)
        if key in self._side and self._side[key].cuda_stream == cur:
            return "side"
        if key in self._aux and self._aux[key].cuda_stream == cur:
            return "aux"
        return "main"

    def _take(self, k, n: int, device, dtype, zeroed: bool = False) -> torch.Tensor:
        cur = self.buf.get(k)
        if cur is not None and cur.numel() >= n:
            return cur
        if _RECORDING:
            raise RuntimeError(
                f"workspace {k[0]!r} ({self.name}) would grow to {n} elements while a launch plan is being "
                f"recorded (earlier recorded launches hold the old buffer): run an uncaptured step of the same "
                f"shapes first")
        alloc = torch.zeros if zeroed else torch.empty
        if self.frozen:
            # a live plan holds buf[k]'s address: this (eager) launch gets a buffer of its own
            e = self._eager.get(k)
            if e is None or e.numel() < n:
                e = alloc(max(n, 1), device=device, dtype=dtype)
                self._eager[k] = e
            return e
        cur = alloc(max(n, 1), device=device, dtype=dtype)
        self.buf[k] = cur
        return cur

    def get(self, key: str, n: int, device, dtype=torch.float32, zeroed: bool = False) -> torch.Tensor:
        """zeroed: a buffer created (or grown) here starts as zeros — for state the kernels keep zero
        between calls themselves (the split-K tile tickets)."""
        if _RECORDING and not self.owned:
            raise RuntimeError("launch-plan recording needs an engine-owned execution context (ops.using)")
        return self._take((key, _dkey(device), dtype, self._role(device)), n, device, dtype, zeroed)

    def fresh(self, key: str, n: int, device, dtype=torch.float32) -> torch.Tensor:
        if not self.owned:   # shared default context: a new allocation (eager use only)
            if _RECORDING:
                raise RuntimeError("launch-plan recording needs an engine-owned execution context (ops.using)")
            return torch.empty(max(n, 1), device=device, dtype=dtype)
        i = self._cursor.get(key, 0)
        self._cursor[key] = i + 1
        return self._take((key, _dkey(device), dtype, ("fresh", i)), n, device, dtype)

    def new_pass(self) -> None:
        self._cursor.clear()

    def tensors(self):
        return list(self.buf.values())


_TLS = threading.local()
_DEFAULT = ExecContext("default", owned=False)
_RECORDING = False


def current() -> ExecContext:
    st = getattr(_TLS, "stack", None)
    return st[-1] if st else _DEFAULT


@contextmanager
def using(ctx: ExecContext):
    """Launches inside run with ``ctx``'s workspaces, streams and device step seed."""
    st = getattr(_TLS, "stack", None)
    if st is None:
        st = _TLS.stack = []
    prev = current()
    st.append(ctx)
    _lib.lib().alignn_set_step_seed(None if ctx.step_seed is None else ctx.step_seed.data_ptr())
    try:
        yield ctx
    finally:
        st.pop()
        _lib.lib().alignn_set_step_seed(None if prev.step_seed is None else prev.step_seed.data_ptr())


@contextmanager
def recording():
    """Marks a launch-plan recording: workspaces may not grow, the default context may not be used."""
    global _RECORDING
    prev = _RECORDING
    _RECORDING = True
    try:
        yield
    finally:
        _RECORDING = prev


def side_stream(device) -> torch.cuda.Stream:
    return current().side(device)


def aux_stream(device) -> torch.cuda.Stream:
    return current().aux(device)


class _WSProxy:
    """``WS.get`` = the current context's workspace (kept for the tools/ scripts)."""

    def get(self, key: str, n: int, device, dtype=torch.float32, zeroed: bool = False) -> torch.Tensor:
        return current().get(key, n, device, dtype, zeroed)


WS = _WSProxy()


def stream_wait(dst: torch.cuda.Stream, src: torch.cuda.Stream) -> None:
    """dst waits for the work queued on src so far (torch's event wait), noted as an ordering
    edge when a launch plan is being recorded (alignn_plan_note_wait)."""
    dst.wait_stream(src)
    check(_lib.lib().alignn_plan_note_wait(dst.cuda_stream, src.cuda_stream), "alignn_plan_note_wait")


def zero_(t: torch.Tensor) -> torch.Tensor:
    """t[...] = 0 by a library kernel (recordable in a launch plan, unlike torch's fill)."""
    _require(t, "zero_")
    if not t.is_contiguous():
        raise ValueError("zero_: contiguous tensors only")
    check(_lib.lib().alignn_fill_f32(t.data_ptr(), t.numel(), 0.0, stream_ptr()), "alignn_fill_f32")
    return t


def add_(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """x += y (contiguous fp32, same element count) by a library kernel (alignn_add_f32)."""
    _require(x, "add_ x")
    _require(y, "add_ y")
    if not (x.is_contiguous() and y.is_contiguous()) or x.numel() != y.numel():
        raise ValueError("add_: contiguous tensors with equal element counts only")
    check(_lib.lib().alignn_add_f32(x.data_ptr(), y.data_ptr(), x.numel(), stream_ptr()), "alignn_add_f32")
    return x


def zeros(*shape, device) -> torch.Tensor:
    return zero_(torch.empty(*shape, device=device))


def copy_(dst: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """dst[...] = src[...] (contiguous fp32, same element count) by a library kernel."""
    _require(dst, "copy_ dst")
    _require(src, "copy_ src")
    if not (dst.is_contiguous() and src.is_contiguous()) or dst.numel() != src.numel():
        raise ValueError("copy_: contiguous tensors with equal element counts only")
    check(_lib.lib().alignn_copy_f32(dst.data_ptr(), src.data_ptr(), dst.numel(), stream_ptr()), "alignn_copy_f32")
    return dst


def copy_many(pairs) -> None:
    """dst.copy_(src) for each (dst, src) pair of same-shape, same-dtype tensors, in one library
    launch per 32 pairs (alignn_copy_many); pairs the kernel cannot take (non-contiguous, misaligned,
    sizes not a multiple of 4 bytes) go through torch's copy."""
    todo = []
    for dst, src in pairs:
        if dst.shape != src.shape or dst.dtype != src.dtype:
            raise ValueError(f"copy_many: {tuple(src.shape)} {src.dtype} into {tuple(dst.shape)} {dst.dtype}")
        nb = src.numel() * src.element_size()
        if nb == 0:
            continue
        if (dst.is_contiguous() and src.is_contiguous() and nb % 4 == 0 and dst.data_ptr() % 16 == 0
                and src.data_ptr() % 16 == 0 and dst.is_cuda and src.is_cuda):
            todo.append((dst.data_ptr(), src.data_ptr(), nb))
        else:
            dst.copy_(src)
    for i in range(0, len(todo), 32):
        chunk = todo[i:i + 32]
        n = len(chunk)
        d = (ctypes.c_void_p * n)(*[c[0] for c in chunk])
        s_ = (ctypes.c_void_p * n)(*[c[1] for c in chunk])
        b = (ctypes.c_int64 * n)(*[c[2] for c in chunk])
        check(_lib.lib().alignn_copy_many(n, s_, d, b, stream_ptr()), "alignn_copy_many")


def clone(src: torch.Tensor) -> torch.Tensor:
    return copy_(torch.empty_like(src, memory_format=torch.contiguous_format), src.contiguous())


# ------------------------------------------------------------------------------------------------
# GEMM
# ------------------------------------------------------------------------------------------------
def _as3(t: torch.Tensor):
    if t.dim() == 2:
        return 1, 0, t.stride(0), t.stride(1), t.size(0), t.size(1)
    if t.dim() == 3:
        return t.size(0), t.stride(0), t.stride(1), t.stride(2), t.size(1), t.size(2)
    raise ValueError("gemm operands must be 2-D or 3-D (batched) views")


GEMM_TRACE: Optional[list] = None
_GEMM_FLAGS = 0       # ORed into AlignnGemmArgs.tile by gemm() (gemm_precision)
GEMM_BF16 = 64        # ALIGNN_GEMM_BF16
GEMM_NOPIPE = 256     # ALIGNN_GEMM_NOPIPE: force the one-stage-in-flight loop (A/B tests)
GEMM_A_BF16, GEMM_B_BF16, GEMM_C_BF16 = 1024, 2048, 4096   # bf16 storage of an operand / the output
GEMM_LDS16 = 16384    # ALIGNN_GEMM_LDS16: bf16 tiled products through bf16 LDS images (forced on; default: A k-contiguous)
GEMM_NOLDS16 = 32768  # ALIGNN_GEMM_NOLDS16: ... forced off (A/B tests)
GEMM_ROWS = 65536     # ALIGNN_GEMM_ROWS: the bf16 row-streaming kernel at any M (tests / A/B)
GEMM_NOROWS = 131072  # ALIGNN_GEMM_NOROWS: ... never
GEMM_NOWGRAD = 262144  # ALIGNN_GEMM_NOWGRAD: the bf16 weight-gradient kernel never (tests / A/B)


@contextmanager
def gemm_precision(precision: str):
    """GEMMs issued inside run with "fp32" (exact fp32 MFMA) or "bf16" arithmetic (bf16-rounded
    inputs on v_mfma_f32_32x32x16_bf16, fp32 accumulation and output: ALIGNN_GEMM_BF16)."""
    global _GEMM_FLAGS
    if precision not in ("fp32", "bf16"):
        raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
    prev = _GEMM_FLAGS
    _GEMM_FLAGS = GEMM_BF16 if precision == "bf16" else 0
    try:
        yield
    finally:
        _GEMM_FLAGS = prev

def set_step_seed(t: Optional[torch.Tensor]) -> None:
    """Register a device int64[1] on the current context that every dropout / jitter kernel launched
    afterwards (in it) mixes into its site seed at run time (alignn_set_step_seed): a recorded plan
    then draws fresh masks on each replay once the caller updates ``t``.  None: host seeds only."""
    if t is not None and (t.dtype != torch.int64 or t.numel() != 1 or not t.is_cuda):
        raise ValueError("step seed must be a device int64 tensor with one element")
    current().step_seed = t
    _lib.lib().alignn_set_step_seed(None if t is None else t.data_ptr())


def gemm(A: torch.Tensor, B: torch.Tensor, C: torch.Tensor, *, alpha: float = 1.0, beta: float = 0.0,
         bias: Optional[torch.Tensor] = None, rowscale: Optional[torch.Tensor] = None,
         bias2: Optional[torch.Tensor] = None, relu: bool = False, mask: Optional[torch.Tensor] = None,
         split_k: Optional[int] = None, reduce_batch: bool = False,
         c_rows: Optional[torch.Tensor] = None, tile: int = 0, path_only: bool = False,
         rowsum: Optional[torch.Tensor] = None):
    """C = act(alpha * A @ B + beta * C + bias + rowscale[:,None] * bias2) [* (mask > 0)].

    A [.., M, K], B [.., K, N], C [.., M, N] are arbitrary strided views (batched when 3-D), fp32 or
    bf16 (bf16 storage, config C3: an operand widened exactly as it is staged, C rounded RNE and
    write-only; bf16 tensors need bf16 arithmetic, gemm_precision("bf16"));
    bias/bias2 [.., N], rowscale [.., M] (strided views too).  ``reduce_batch``: A/B batched, C is
    2-D and receives the sum over the batch (K must be a multiple of 16).  ``c_rows`` (int32 [M]):
    logical row r of C is stored at C[c_rows[r]] (C then has any number of rows >= max index).
    ``rowsum`` (fp32 contiguous [M]): also rowsum[m] = sum_k A[m, k] from the same launch — the bias
    gradient beside a weight gradient dW = dY^T X (A = dY^T), instead of a colsum pass over dY."""
    ba, sab, sam, sak, M, K = _as3(A)
    bb, sbb, sbk, sbn, K2, N = _as3(B)
    bc, scb, scm, scn, M2, N2 = _as3(C)
    if c_rows is not None:
        if c_rows.dtype != torch.int32 or c_rows.numel() != M:
            raise ValueError("gemm: c_rows must be int32 with M entries")
        M2 = M
    batch = max(ba, bb, bc)
    if reduce_batch:
        if bc != 1 or K2 != K or M2 != M or N2 != N or ba not in (1, batch) or bb not in (1, batch):
            raise ValueError(f"gemm(reduce_batch) shape mismatch: A{tuple(A.shape)} B{tuple(B.shape)} C{tuple(C.shape)}")
    elif K2 != K or M2 != M or N2 != N or bc != batch or ba not in (1, batch) or bb not in (1, batch):
        raise ValueError(f"gemm shape mismatch: A{tuple(A.shape)} B{tuple(B.shape)} C{tuple(C.shape)}")
    a = GemmArgs()
    a.M, a.N, a.K, a.batch = M, N, K, batch
    a.A, a.sam, a.sak, a.sab = A.data_ptr(), sam, sak, (sab if ba > 1 else 0)
    a.B, a.sbk, a.sbn, a.sbb = B.data_ptr(), sbk, sbn, (sbb if bb > 1 else 0)
    a.C, a.scm, a.scn, a.scb = C.data_ptr(), scm, scn, (scb if bc > 1 else 0)
    if bias is not None:
        a.bias = bias.data_ptr()
        a.sbias_b = bias.stride(0) if bias.dim() == 2 else 0
    if rowscale is not None:
        if bias2 is None:
            raise ValueError("rowscale needs bias2")
        a.rowscale = rowscale.data_ptr()
        a.srs_m = rowscale.stride(-1)
        a.srs_b = rowscale.stride(0) if rowscale.dim() == 2 else 0
        a.bias2 = bias2.data_ptr()
        a.sb2_b = bias2.stride(0) if bias2.dim() == 2 else 0
    if mask is not None:
        a.mask, a.smk_m, a.smk_n = mask.data_ptr(), mask.stride(0), mask.stride(1)
    a.alpha, a.beta, a.relu = float(alpha), float(beta), int(bool(relu))
    a.reduce_batch = int(bool(reduce_batch) and batch > 1)
    if c_rows is not None:
        a.c_rows = c_rows.data_ptr()
    if rowsum is not None:
        if (rowsum.dtype != torch.float32 or rowsum.numel() != M or not rowsum.is_contiguous() or batch != 1
                or reduce_batch):
            raise ValueError("gemm: rowsum must be a contiguous fp32 [M] tensor (batch 1, no reduce_batch)")
        a.rowsum = rowsum.data_ptr()
    a.split_k = 0 if split_k is None else int(split_k)   # 0: the library plans tile shape and split-K
    io = 0
    for t, flag in ((A, GEMM_A_BF16), (B, GEMM_B_BF16), (C, GEMM_C_BF16)):
        if t.dtype == torch.bfloat16:
            io |= flag
        elif t.dtype != torch.float32:
            raise TypeError(f"gemm: operands must be float32 or bfloat16, got {t.dtype}")
    if io and not ((_GEMM_FLAGS | int(tile)) & GEMM_BF16):
        raise ValueError("gemm: bf16 operands need bf16 arithmetic (ops.gemm_precision('bf16'))")
    a.tile = int(tile) | _GEMM_FLAGS | io
    if path_only:   # the kernel the library takes (0 tiled, 2 bf16 row-streaming, 3 bf16 weight-gradient);
        #             nothing runs
        return int(_lib.lib().alignn_gemm_path(ctypes.byref(a)))
    need = int(_lib.lib().alignn_gemm_workspace(ctypes.byref(a)))
    if need < 0:
        raise ValueError("gemm: invalid shape")
    if need > 0:
        ws = WS.get("gemm", need, C.device)
        a.workspace, a.workspace_elems = ws.data_ptr(), ws.numel()
    if GEMM_TRACE is not None:   # tuning hook (tools/gemm_bench.py): record the call's operands
        GEMM_TRACE.append(dict(A=A, B=B, C=C, alpha=alpha, beta=beta, bias=bias, rowscale=rowscale, bias2=bias2,
                               relu=relu, mask=mask, reduce_batch=reduce_batch, c_rows=c_rows, rowsum=rowsum))
    key = f"gemm_f32 M{M} N{N} K{K} b{batch}" + "".join(f" {n}16" for t, n in ((A, "A"), (B, "B"), (C, "C"))
                                                      if t.dtype == torch.bfloat16)
    if profiling.active(key) or profiling.active("*gemm"):
        nbytes = batch * (A.element_size() * M * K + B.element_size() * K * N
                          + C.element_size() * M * N * (2 if beta else 1))
        profiling.launch(key, 2.0 * M * N * K * batch, nbytes,
                         lambda: check(_lib.lib().alignn_gemm_f32(ctypes.byref(a), stream_ptr()), "alignn_gemm_f32"))
    else:
        check(_lib.lib().alignn_gemm_f32(ctypes.byref(a), stream_ptr()), "alignn_gemm_f32")
    return C


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor], out: Optional[torch.Tensor] = None,
           relu: bool = False) -> torch.Tensor:
    """out = x @ w.T + b (nn.Linear)."""
    if out is None:
        out = torch.empty(x.size(0), w.size(0), device=x.device, dtype=x.dtype)
    return gemm(x, w.t(), out, bias=b, relu=relu)


def colsum(X: torch.Tensor, out: torch.Tensor, accumulate: bool = False) -> torch.Tensor:
    """out (+)= X.sum(0) (fp32 sums of fp32 or bf16 rows)."""
    M, N = X.shape
    if X.stride(1) != 1:
        raise ValueError("colsum: rows must be unit-stride")
    ws = WS.get("colsum", 256 * N, X.device)
    fn = _lib.lib().alignn_colsum_bf16 if X.dtype == torch.bfloat16 else _lib.lib().alignn_colsum_f32
    check(fn(X.data_ptr(), M, N, X.stride(0), out.data_ptr(), int(accumulate), ws.data_ptr(), stream_ptr()),
          "alignn_colsum")
    return out


def wcolsum2(X1: torch.Tensor, W1: torch.Tensor, X2: torch.Tensor, W2: torch.Tensor, out: torch.Tensor,
             accumulate: bool = False) -> torch.Tensor:
    """out[j] (+)= sum_r W1[r, j // C] X1[r, j] + W2[r, j // C] X2[r, j], C = N // W1.size(1): the
    per-head w-bar gradient sum_n Q_nh sigz_nh + dout_nh sumA_nh (alignn_wcolsum2_f32)."""
    M, N = X1.shape
    Hh = W1.size(1)
    if (tuple(X2.shape) != (M, N) or tuple(W1.shape) != (M, Hh) or tuple(W2.shape) != (M, Hh) or N % Hh
            or X1.stride(1) != 1 or X2.stride(1) != 1 or W1.stride(1) != 1 or W2.stride(1) != 1 or out.numel() != N
            or not out.is_contiguous()):
        raise ValueError("wcolsum2: inconsistent shapes or strides")
    ws = WS.get("colsum", 256 * N, X1.device)
    check(_lib.lib().alignn_wcolsum2_f32(M, N, N // Hh, X1.data_ptr(), X1.stride(0), W1.data_ptr(), W1.stride(0),
                                         X2.data_ptr(), X2.stride(0), W2.data_ptr(), W2.stride(0), out.data_ptr(),
                                         int(accumulate), ws.data_ptr(), stream_ptr()), "alignn_wcolsum2_f32")
    return out


SMALLK_MAX = 16   # alignn_linear_smallk_f32: K <= 16
SMALLN_MAX = 16   # alignn_gemm_tn_smalln_f32: N <= 16


def linear_smallk_ok(X: torch.Tensor, W: torch.Tensor, out: torch.Tensor) -> bool:
    """Shapes alignn_linear_smallk_f32 takes (else use gemm)."""
    return (X.dim() == 2 and X.stride(1) == 1 and W.dim() == 2 and W.stride(1) == 1 and out.stride(1) == 1
            and W.size(1) == X.size(1) <= SMALLK_MAX and out.size(1) == W.size(0) and out.size(0) == X.size(0)
            and W.size(0) % 4 == 0 and out.stride(0) % 4 == 0 and out.data_ptr() % 16 == 0)


def linear_smallk(X: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], out: torch.Tensor,
                  relu: bool = False) -> torch.Tensor:
    """out = act(X W^T + bias) for K = X.size(1) <= 16, streamed (HBM-bound) instead of tiled."""
    if not linear_smallk_ok(X, W, out):
        raise ValueError(f"linear_smallk: unsupported shapes X{tuple(X.shape)} W{tuple(W.shape)} out{tuple(out.shape)}")
    check(_lib.lib().alignn_linear_smallk_f32(X.data_ptr(), X.stride(0), X.size(0), X.size(1), W.data_ptr(),
                                              W.stride(0), None if bias is None else bias.data_ptr(), W.size(0),
                                              int(bool(relu)), out.data_ptr(), out.stride(0), stream_ptr()),
          "alignn_linear_smallk_f32")
    return out


SMALLK_BF16_MAX = 15   # alignn_linear_smallk_bf16out: K + the bias column within one 16-deep MFMA k step


def linear_smallk_bf16_ok(X: torch.Tensor, W: torch.Tensor, out: torch.Tensor) -> bool:
    """Shapes alignn_linear_smallk_bf16out takes: 1 <= K <= 15, N % 32 == 0, N <= 1024, unit inner
    strides, 16-byte aligned output rows."""
    return (out.dtype == torch.bfloat16 and X.dim() == 2 and X.stride(1) == 1 and W.dim() == 2 and W.stride(1) == 1
            and out.stride(1) == 1 and 1 <= W.size(1) == X.size(1) <= SMALLK_BF16_MAX and out.size(1) == W.size(0)
            and out.size(0) == X.size(0) and W.size(0) % 32 == 0 and W.size(0) <= 1024 and out.stride(0) % 8 == 0
            and out.data_ptr() % 16 == 0)


def linear_smallk_bf16(X: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], out: torch.Tensor,
                       relu: bool = False) -> torch.Tensor:
    """out (bf16) = act(bf16(bf16(X) bf16(W)^T + bf16(bias))) — a Linear under bf16 autocast (fp32
    accumulation on the matrix cores, ReLU on the rounded output), the arithmetic of the deferred encoder
    backward's recomputed mask (alignn_enc_bwd_bf16 without F) bit for bit."""
    if not linear_smallk_bf16_ok(X, W, out):
        raise ValueError(f"linear_smallk_bf16: unsupported shapes X{tuple(X.shape)} W{tuple(W.shape)} "
                         f"out{tuple(out.shape)} {out.dtype}")
    check(_lib.lib().alignn_linear_smallk_bf16out(X.data_ptr(), X.stride(0), X.size(0), X.size(1), W.data_ptr(),
                                                  W.stride(0), None if bias is None else bias.data_ptr(), W.size(0),
                                                  int(bool(relu)), out.data_ptr(), out.stride(0), stream_ptr()),
          "alignn_linear_smallk_bf16out")
    return out


def gemm_tn_smalln(A: torch.Tensor, X: torch.Tensor, C: torch.Tensor, colsum: Optional[torch.Tensor] = None,
                   accumulate: bool = False) -> torch.Tensor:
    """C (+)= A^T X and colsum (+)= A.sum(0) in one pass over A [K, M] (X [K, N], N <= 16): the
    weight and bias gradients of a Linear with few inputs."""
    K, M = A.shape
    N = X.size(1)
    if (A.stride(1) != 1 or X.stride(1) != 1 or C.stride(1) != 1 or X.size(0) != K or tuple(C.shape) != (M, N)
            or N > SMALLN_MAX or (colsum is not None and (colsum.numel() != M or not colsum.is_contiguous()))):
        raise ValueError(f"gemm_tn_smalln: unsupported shapes A{tuple(A.shape)} X{tuple(X.shape)} C{tuple(C.shape)}")
    lib = _lib.lib()
    need = int(lib.alignn_gemm_tn_smalln_workspace(K, M, N))
    ws = WS.get("smalln", need, A.device)
    check(lib.alignn_gemm_tn_smalln_f32(A.data_ptr(), A.stride(0), K, M, X.data_ptr(), X.stride(0), N, C.data_ptr(),
                                        C.stride(0), None if colsum is None else colsum.data_ptr(), int(accumulate),
                                        ws.data_ptr(), ws.numel(), stream_ptr()), "alignn_gemm_tn_smalln_f32")
    return C


ENC_XF_KMAX = 12   # alignn_enc_bwd_bf16 without the stored layer: kin + the bias column <= 16 (one k step)


def enc_bwd_ok(D: int, H: int, L: int, kin: int) -> bool:
    """Shapes alignn_enc_bwd_f32 takes (else the per-layer dF path)."""
    return (0 < D <= 256 and D % 4 == 0 and 0 <= kin <= 16 and 1 <= L <= _lib.ENCBWD_MAX_LAYERS and H in (1, 2, 4, 8)
            and H * L <= 16)


def enc_bwd(g: "GraphCSR", x: torch.Tensor, W1: torch.Tensor, b1: torch.Tensor, Us, Vds, dzs, alphas,
            dW1: torch.Tensor, db1: torch.Tensor, accumulate: bool = False,
            F: Optional[torch.Tensor] = None, bf16: bool = False) -> None:
    """Deferred backward of the angle encoder's first Linear + ReLU over the line graph ``g``:
    dW1/db1 (+)= sum_t dpre_t x_t^T / dpre_t with dpre_t = relu'(W1 x_t + b1) * sum_l,h
    (dz_l u_l + alpha_l Vd_l) — see include/alignn_hip.h (alignn_enc_bwd_f32).  F: the forward's bf16
    hidden layer [T, 256] (bf16 storage, config C3) — the two products then run on the matrix cores in
    bf16 with the ReLU mask read from F (alignn_enc_bwd_bf16).  bf16 without F: the same products with
    the mask recomputed from x (the line convs' recompute path, alignn_lg_fwd_x)."""
    L = len(Us)
    T, kin = x.shape
    D = W1.size(0)
    H = Us[0].size(1) if L else 1
    if (not enc_bwd_ok(D, H, L, kin) or len(Vds) != L or len(dzs) != L or len(alphas) != L or T != g.m
            or x.stride(1) != 1 or not W1.is_contiguous() or tuple(W1.shape) != (D, kin) or not dW1.is_contiguous()
            or tuple(dW1.shape) != (D, kin) or b1.numel() != D or db1.numel() != D):
        raise ValueError("enc_bwd: unsupported or inconsistent shapes")
    for U, Vd, dz, al in zip(Us, Vds, dzs, alphas):
        if (tuple(U.shape) != (g.n, H, D) or tuple(Vd.shape) != (g.n, H, D) or not U.is_contiguous()
                or not Vd.is_contiguous() or dz.size(0) < T or al.size(0) < T or dz.size(-1) != H
                or al.size(-1) != H or not dz.is_contiguous() or not al.is_contiguous()):
            raise ValueError("enc_bwd: per-layer operand does not cover the graph")
    lib = _lib.lib()
    a = _lib.EncBwdArgs()
    a.n, a.T, a.D, a.H, a.L, a.kin = g.n, T, D, H, L, kin
    a.dst_at = g.dst_at.data_ptr()
    a.off_dst = g.off_dst.data_ptr()
    a.x, a.ldx = x.data_ptr(), x.stride(0)
    a.w1, a.b1 = W1.data_ptr(), b1.data_ptr()
    for l in range(L):
        a.U[l], a.Vd[l] = Us[l].data_ptr(), Vds[l].data_ptr()
        a.dz[l], a.alpha[l] = dzs[l].data_ptr(), alphas[l].data_ptr()
    a.dW1, a.db1, a.accumulate = dW1.data_ptr(), db1.data_ptr(), int(bool(accumulate))
    need = int(lib.alignn_enc_bwd_workspace(D, kin))
    ws = WS.get("enc_bwd", need, x.device)
    a.workspace, a.workspace_elems = ws.data_ptr(), ws.numel()
    # compulsory bytes: x rows, targets, 2LH scalars per edge; U/Vd rows once per target
    nbytes = 4.0 * (T * (kin + 1 + 2 * L * H) + 2 * L * g.n * H * D)
    if bf16 and F is None:
        if D != 256 or H % 2 or kin < 1 or kin > 12:
            raise ValueError("enc_bwd: the bf16 recompute form needs D = 256, H even, 1 <= kin <= 12")
        profiling.launch(f"enc_bwd_bf16 T{T} L{L} x", 0.0, nbytes,
                         lambda: check(lib.alignn_enc_bwd_bf16(ctypes.byref(a), None, 0, stream_ptr()),
                                       "alignn_enc_bwd_bf16"))
        return
    if F is not None:
        if (F.dtype != torch.bfloat16 or F.dim() != 2 or F.size(0) < T or F.size(1) != D or F.stride(1) != 1
                or F.stride(0) % 8 or F.data_ptr() % 16 or D != 256 or H % 2 or kin < 1):
            raise ValueError("enc_bwd: F must be the bf16 [T, 256] hidden layer, rows 16-byte aligned "
                             "(and H even, kin >= 1)")
        nbytes += 2.0 * T * D
        profiling.launch(f"enc_bwd_bf16 T{T} L{L}", 0.0, nbytes,
                         lambda: check(lib.alignn_enc_bwd_bf16(ctypes.byref(a), F.data_ptr(), F.stride(0),
                                                               stream_ptr()), "alignn_enc_bwd_bf16"))
        return
    profiling.launch(f"enc_bwd T{T} L{L}", 0.0, nbytes,
                     lambda: check(lib.alignn_enc_bwd_f32(ctypes.byref(a), stream_ptr()), "alignn_enc_bwd_f32"))


# ------------------------------------------------------------------------------------------------
# Graph preparation
# ------------------------------------------------------------------------------------------------
class GraphCSR:
    """Target- and source-sorted CSR of one edge_index (see include/alignn_hip.h)."""

    __slots__ = ("n", "m", "off_dst", "perm_dst", "src_at", "dst_at", "off_src", "pos_src", "err", "_sched", "rows",
                 "n_full", "cmap", "_dst_src", "xcd_chunk", "policy", "deg_bound")

    # in-degree above which a target node gets a 4-wave workgroup (LDS merge of the waves); below it
    # one wave walks the node's edges.  256: every node of the MP-like line graph (in-degree <= 132
    # under the PyG offset rule) takes the 1-wave path — measured +6.2 % step at B = 32, +8.7 % at
    # B = 256 bf16 vs 32 (line bwd_dst 194 -> 159 us; profiles/r01/v27_sweep_heavy_threshold.log)
    def __init__(self, edge_index: torch.Tensor, n: int, policy: Optional["SchedulePolicy"] = None):
        if edge_index.dtype != torch.int64 or edge_index.dim() != 2 or edge_index.size(0) != 2:
            raise ValueError("edge_index must be int64 [2, m]")
        ei = edge_index.contiguous()
        dev = ei.device
        m = ei.size(1)
        self.n, self.m = n, m
        i32 = dict(device=dev, dtype=torch.int32)
        self.off_dst = torch.empty(n + 1, **i32)
        self.perm_dst = torch.empty(max(m, 1), **i32)
        self.src_at = torch.empty(max(m, 1), **i32)
        self.dst_at = torch.empty(max(m, 1), **i32)
        self.off_src = torch.empty(n + 1, **i32)
        self.pos_src = torch.empty(max(m, 1), **i32)
        self.err = torch.zeros(1, **i32)
        self._sched = None
        self._dst_src = None
        self.policy = DEFAULT_SCHEDULE if policy is None else policy
        self.xcd_chunk = 1   # work items per workgroup of the kernels that read this graph's list
        self.rows = None     # compacted graph: int32 ids of its nodes in the full node set
        self.n_full = n
        self.cmap = None     # compacted graph: int32 [n_full] full row -> node id, -1 if inactive
        self.deg_bound = None   # host bound of every in-degree (store batches): device-built schedule
        ws = WS.get("graph", 2 * n + 64, dev, torch.int32)
        check(_lib.lib().alignn_graph_prep(ei.data_ptr(), m, n, self.off_dst.data_ptr(), self.perm_dst.data_ptr(),
                                           self.src_at.data_ptr(), self.dst_at.data_ptr(), self.off_src.data_ptr(),
                                           self.pos_src.data_ptr(), ws.data_ptr(), self.err.data_ptr(),
                                           stream_ptr()), "alignn_graph_prep")

    def dst_src(self) -> torch.Tensor:
        """Targets in by-source order, dst_at[pos_src[i]] (int32 [m]; built once per graph)."""
        if self._dst_src is None:
            if _RECORDING:
                raise RuntimeError("GraphCSR.dst_src built during a launch-plan recording: prepare the batch first")
            self._dst_src = self.dst_at[self.pos_src.long()].contiguous() if self.m else self.dst_at[:0].clone()
        return self._dst_src

    def schedule(self, deg: Optional[np.ndarray] = None):
        """Light/heavy target-node lists for the attention kernels (host-built once per graph:
        one small device->host copy of the offsets — or the in-degrees ``deg`` the caller fetched —
        numpy ordering, one upload)."""
        if self._sched is None and deg is None and self.device_schedule_ok():
            self._sched = self._schedule_on_device()
        if self._sched is None:
            if deg is None:
                off = self.off_dst.cpu().numpy().astype(np.int64)
                deg = off[1:] - off[:-1] if self.n else np.zeros(0, np.int64)
            po = self.policy
            light, heavy = schedule_lists(deg, po.heavy_threshold, po.wave_items, po.xcd_items and po.wave_items,
                                          po.xcds, self.xcd_chunk)
            both = torch.from_numpy(np.concatenate([light, heavy]).astype(np.int32)).to(self.off_dst.device)
            light, heavy = both[:len(light)], both[len(light):]
            sc = _lib.Schedule()
            sc.light, sc.n_light = (light.data_ptr() if light.numel() else None), light.numel()
            sc.heavy, sc.n_heavy = (heavy.data_ptr() if heavy.numel() else None), heavy.numel()
            sc.flags = _lib.SCHED_WAVE_ITEMS if po.wave_items else 0
            self._sched = (sc, light, heavy)
        return self._sched[0]

    def device_schedule_ok(self) -> bool:
        """The work list can be built on the device (alignn_schedule_build, no host round trip): the
        caller bounded every in-degree on the host (deg_bound) below the heavy threshold — so there is
        no heavy list and the light list holds all n targets — and the policy orders by degree."""
        po = self.policy
        return (self.deg_bound is not None and po.wave_items and 0 <= self.deg_bound <= po.heavy_threshold
                and po.heavy_threshold <= 512 and po.xcds <= 8)

    def _schedule_on_device(self):
        po = self.policy
        light = torch.empty(max(self.n, 1), dtype=torch.int32, device=self.off_dst.device)[:self.n]
        check(_lib.lib().alignn_schedule_build(self.off_dst.data_ptr(), self.n, po.heavy_threshold,
                                               po.xcds if po.xcd_items else 1, max(1, int(self.xcd_chunk)),
                                               light.data_ptr() if self.n else None, self.err.data_ptr(),
                                               stream_ptr()), "alignn_schedule_build")
        heavy = light[:0]
        sc = _lib.Schedule()
        sc.light, sc.n_light = (light.data_ptr() if self.n else None), self.n
        sc.heavy, sc.n_heavy = None, 0
        sc.flags = _lib.SCHED_WAVE_ITEMS if po.wave_items else 0
        return (sc, light, heavy)

    def family(self, D: int, H: int, F: Optional[torch.Tensor], feat_row: Optional[torch.Tensor] = None) -> int:
        """Attention kernel family the library runs for this graph and operands (3: single-wave
        items, lgconv.hip; 2: light/heavy workgroups, tconv.hip); alignn_tconv_family.  bf16 feature
        rows (alignn_tconv_fwd_ex) always take family 2."""
        if F is not None and F.dtype == torch.bfloat16:
            return 2
        return int(_lib.lib().alignn_tconv_family(D, H, None if feat_row is None else feat_row.data_ptr(),
                                                   None if F is None else F.data_ptr(), ctypes.byref(self.schedule())))

    def check_indices(self, what: str) -> None:
        """Host check of the device error flag (one sync).  PyG raises IndexError here."""
        err = int(self.err.item())
        if err & 1:
            raise IndexError(f"{what}: edge index out of range [0, {self.n})")
        if err & 2:
            raise RuntimeError(f"{what}: an in-degree exceeds the host bound the device schedule was built for")


@dataclass(frozen=True)
class SchedulePolicy:
    """How GraphCSR.schedule() lays out the attention kernels' work items — fixed per graph at
    construction (an immutable value: two trainers in one process never share mutable switches).

    heavy_threshold: in-degree above which a target node gets a 4-wave workgroup (LDS merge of the
    waves); below it one wave walks the node's edges.  256: every node of the MP-like line graph
    (in-degree <= 132 under the PyG offset rule) takes the 1-wave path — measured +6.2 % step at
    B = 32, +8.7 % at B = 256 bf16 vs 32 (profiles/r01/v27_sweep_heavy_threshold.log).
    wave_items: every target a single-wave work item, longest in-edge list first (lgconv.hip, the
    D = 256 line-graph kernels; other calls keep tconv.hip's light/heavy kernels).
    xcd_items: work items interleaved so that XCD x (workgroup i runs on XCD i % 8) walks the x-th
    contiguous range of target ids, ranges of equal EDGE count, longest first within each: a
    target's sources lie near it (PyG's per-graph index windows), so each XCD's L2 holds the K/V
    rows its gathers need (line-graph bwd_dst fetch 588 -> 300 MB per launch; step +1.8 % at B = 32,
    profiles/r02/v24_ab_xcd_items_edge_balanced.log)."""
    heavy_threshold: int = 256
    wave_items: bool = True
    xcd_items: bool = True
    xcds: int = 8


DEFAULT_SCHEDULE = SchedulePolicy()


def schedule_lists(deg: np.ndarray, heavy_threshold: int, by_degree: bool, xcd_ranges: bool, xcds: int = 8,
                   chunk: int = 1):
    """(light, heavy) work lists of target ids for the attention kernels, from the in-degrees.

    light: targets with in-degree 1..heavy_threshold, then the in-degree-0 ones (the kernels skip
    per-workgroup setup for items that start with an empty node); heavy: in-degree above it.
    by_degree: longest segments first (their waves start in the first round of resident workgroups;
    each node is still one wave's work, so results do not change).  xcd_ranges: the light targets
    with in-edges split into ``xcds`` contiguous id ranges holding equal numbers of EDGES (a target's
    sources lie near it, so XCD x, which runs workgroups i % xcds == x, keeps the K/V rows of its
    range in its own L2; equal target counts put 322 132-edge targets on one XCD's 256 wave slots),
    longest first within each range, and interleaved range by range in chunks of ``chunk`` items
    (kernels taking several items per workgroup keep one workgroup's items in one range)."""
    n = len(deg)
    idx = np.arange(n, dtype=np.int64)
    light_m = deg <= heavy_threshold
    lit = idx[light_m & (deg > 0)]
    hv = idx[~light_m]
    if by_degree:
        lit = lit[np.argsort(-deg[lit], kind="stable")]
        hv = hv[np.argsort(-deg[hv], kind="stable")]
    if xcd_ranges and len(lit) > xcds:
        cum = np.cumsum(deg)
        tot = int(cum[-1]) if n else 0
        bounds = np.asarray([0] + [int(np.searchsorted(cum, tot * x // xcds, side="right")) for x in range(1, xcds)]
                            + [n])
        xr = np.searchsorted(bounds, lit, side="right") - 1          # range of each target
        perm = np.argsort(xr, kind="stable")                           # by range, keeping the lit order
        start = np.searchsorted(xr[perm], np.arange(xcds))
        rank = np.empty(len(lit), np.int64)
        rank[perm] = np.arange(len(lit)) - start[xr[perm]]             # position within its range
        c = max(1, int(chunk))
        lit = lit[np.lexsort((rank % c, xr, rank // c))]               # chunk j of range 0, 1, ..., then j + 1
    return np.concatenate([lit, idx[light_m & (deg == 0)]]), hv


def gather_rows(src: torch.Tensor, idx: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    rows = idx.numel()
    cols = src.size(1)
    if out is None:
        out = torch.empty(rows, cols, device=src.device, dtype=src.dtype)
    check(_lib.lib().alignn_gather_rows_f32(src.data_ptr(), src.stride(0), idx.data_ptr(), rows, cols,
                                            out.data_ptr(), out.stride(0), stream_ptr()), "alignn_gather_rows_f32")
    return out


# ------------------------------------------------------------------------------------------------
# TransformerConv attention
# ------------------------------------------------------------------------------------------------
def scatter_rows(src: torch.Tensor, idx: torch.Tensor, out: torch.Tensor, accumulate: bool = False) -> torch.Tensor:
    """out[idx[i]] (+)= src[i] (idx: distinct int32 row indices)."""
    if idx.dtype != torch.int32 or src.size(0) != idx.numel() or src.size(1) != out.size(1):
        raise ValueError("scatter_rows: idx must be int32 with one entry per source row, equal widths")
    check(_lib.lib().alignn_scatter_rows_f32(src.data_ptr(), src.stride(0), idx.data_ptr(), idx.numel(), src.size(1),
                                             out.data_ptr(), out.stride(0), int(bool(accumulate)), stream_ptr()),
          "alignn_scatter_rows_f32")
    return out


def _tconv_bytes(n: int, m: int, D: int, H: int, kind: str, dF_rw: int = 1, f_elem: int = 4) -> float:
    """Compulsory HBM bytes of one launch (every operand touched once, ideal caching).
    dF_rw: [m, D] edge-feature gradient rows moved by bwd_dst (0 none, 1 written, 2 read + written).
    f_elem: bytes per edge-feature element read (2: bf16 rows)."""
    f = 4.0
    feat = m * D * f_elem / 4.0
    if kind == "fwd":   # Q,K,V + U + edge features + CSR in; aggV + S + 3 stats out
        return f * (3 * n * D + n * H * D + feat + 2 * m + n + n * D + n * H * D + 3 * n * H)
    if kind == "bwd_dst":  # Q,K,V,U,Vd,dout,outp,features,stats in; dQ,Sz,sigz,dz,alpha(,dF) out
        return f * (3 * n * D + 2 * n * H * D + 2 * n * D + feat + 2 * n * H + 2 * m + n
                    + n * D + n * H * D + n * H + 2 * m * H + dF_rw * m * D)
    return f * (2 * n * D + 2 * m * H + 2 * m + n + 2 * n * D)  # bwd_src


def _check_tconv(g: GraphCSR, D: int, H: int, QKVR, F, feat_row, node_out=(), node_heads=(), edge_heads=()):
    """Host check that every operand covers what the kernels index (n target/source rows, m edge
    rows) before a launch: an undersized buffer would be an out-of-bounds device access."""
    n, m = g.n, g.m
    if QKVR.size(0) < n or QKVR.size(1) < 3 * D or QKVR.stride(1) != 1:
        raise ValueError(f"tconv: QKVR {tuple(QKVR.shape)} must cover [{n}, >= {3 * D}] row-major")
    if F is None or F.size(1) < D or F.stride(1) != 1:
        raise ValueError("tconv: edge features F [m, D] row-major required")
    if m > 0 and F.size(0) < (m if feat_row is None else int(feat_row.numel())):
        raise ValueError(f"tconv: F has {F.size(0)} rows, the graph has {m} edges")
    if feat_row is not None and feat_row.numel() < m:
        raise ValueError("tconv: feat_row must have one entry per edge")
    for t in node_out:
        if t is not None and t.numel() < n * D:
            raise ValueError(f"tconv: per-node operand {tuple(t.shape)} smaller than [{n}, {D}]")
    for t in node_heads:
        if t is not None and t.numel() < n * H:
            raise ValueError(f"tconv: per-node stats {tuple(t.shape)} smaller than [{n}, {H}]")
    for t in edge_heads:
        if t is not None and t.numel() < m * H:
            raise ValueError(f"tconv: per-edge stats {tuple(t.shape)} smaller than [{m}, {H}]")


def tconv_fwd(g: GraphCSR, D: int, H: int, QKVR: torch.Tensor, U: torch.Tensor, wbar: Optional[torch.Tensor],
              F: Optional[torch.Tensor], feat_row: Optional[torch.Tensor], aggV, S, sumA, mstat, den, drop_p: float,
              seed: int):
    """F: fp32 edge-feature rows, or bf16 (config C3: the atom graph's bond state as autocast casts it)."""
    _check_tconv(g, D, H, QKVR, F, feat_row, node_out=(aggV,), node_heads=(sumA, mstat, den))
    if U.numel() < g.n * H * D or S.numel() < g.n * H * D:
        raise ValueError("tconv_fwd: U and S must be [n, H, D]")
    fbf = F is not None and F.dtype == torch.bfloat16
    profiling.launch(f"tconv_fwd n{g.n} m{g.m}" + (" F16" if fbf else ""), 0.0,
                     _tconv_bytes(g.n, g.m, D, H, "fwd", f_elem=2 if fbf else 4),
                     lambda: check(_lib.lib().alignn_tconv_fwd_ex(
                         g.n, g.m, D, H, g.off_dst.data_ptr(), g.src_at.data_ptr(), _p(feat_row),
                         ctypes.byref(g.schedule()), QKVR.data_ptr(), QKVR.stride(0), U.data_ptr(), _p(wbar),
                         _p(F), 0 if F is None else F.stride(0), int(fbf), aggV.data_ptr(), S.data_ptr(),
                         sumA.data_ptr(), mstat.data_ptr(), den.data_ptr(), float(drop_p), int(seed) & (2**64 - 1),
                         stream_ptr()), "alignn_tconv_fwd"))


def tconv_bwd_dst(g: GraphCSR, D: int, H: int, QKVR, U, Vd, wbar, F, feat_row, dout, outp, mstat, den,
                  dq, Sz, sigz, dz_e, alpha_e, dF, accumulate_dF: int, drop_p: float, seed: int):
    """accumulate_dF: bit 0 add into dF, bit 1 apply the ReLU mask (F > 0) to the result.  dF None:
    no edge-feature gradient (the line graph's deferred angle-encoder backward, ops.enc_bwd)."""
    _check_tconv(g, D, H, QKVR, F, feat_row, node_out=(dout, outp), node_heads=(mstat, den, sigz),
                 edge_heads=(dz_e, alpha_e))
    if U.numel() < g.n * H * D or Vd.numel() < g.n * H * D or Sz.numel() < g.n * H * D or dq.size(0) < g.n:
        raise ValueError("tconv_bwd_dst: U, Vd, Sz must be [n, H, D] and dq [n, >= D]")
    if dF is not None and dF.size(0) < F.size(0):
        raise ValueError("tconv_bwd_dst: dF must cover the rows of F")
    if dF is not None and dF.dtype == torch.bfloat16:
        # bf16 storage: the edge features' gradient as autocast's bf16 cast returns it (write-only)
        if accumulate_dF & 1:
            raise ValueError("tconv_bwd_dst: a bf16 dF is written, not accumulated")
        accumulate_dF = int(accumulate_dF) | 4
    fbf = F is not None and F.dtype == torch.bfloat16
    profiling.launch(f"tconv_bwd_dst n{g.n} m{g.m}" + (" F16" if fbf else ""), 0.0,
                     _tconv_bytes(g.n, g.m, D, H, "bwd_dst", 0 if dF is None else (2 if accumulate_dF & 1 else 1),
                                  f_elem=2 if fbf else 4),
                     lambda: check(_lib.lib().alignn_tconv_bwd_dst_ex(
                         g.n, g.m, D, H, g.off_dst.data_ptr(), g.src_at.data_ptr(), _p(feat_row),
                         ctypes.byref(g.schedule()), QKVR.data_ptr(), QKVR.stride(0),
                         U.data_ptr(), Vd.data_ptr(), _p(wbar), _p(F), 0 if F is None else F.stride(0), int(fbf),
                         dout.data_ptr(), outp.data_ptr(),
                         mstat.data_ptr(), den.data_ptr(), dq.data_ptr(), dq.stride(0), Sz.data_ptr(),
                         sigz.data_ptr(), dz_e.data_ptr(), alpha_e.data_ptr(), _p(dF),
                         0 if dF is None else dF.stride(0), int(accumulate_dF), float(drop_p),
                         int(seed) & (2**64 - 1), stream_ptr()), "alignn_tconv_bwd_dst"))


def _lg_bf16_bytes(n: int, m: int, D: int, H: int, kind: str) -> float:
    """Compulsory HBM bytes of one bf16-storage launch: K|V and the edge-feature rows at 2 bytes,
    everything else fp32 (as _tconv_bytes)."""
    if kind == "fwd":   # Q (4) + K,V (2) + U + features (2) + CSR in; aggV + S + 3 stats out
        return 4.0 * (n * D + n * H * D + 2 * m + n + n * D + n * H * D + 3 * n * H) + 2.0 * (2 * n * D + m * D)
    # bwd_dst: Q,U,Vd,dout,outp,stats,CSR in (4) + K,V,features (2); dQ,Sz,sigz,dz,alpha out
    return (4.0 * (n * D + 2 * n * H * D + 2 * n * D + 2 * n * H + 2 * m + n + n * D + n * H * D + n * H + 2 * m * H)
            + 2.0 * (2 * n * D + m * D))


def _check_lg_bf16(g: GraphCSR, D: int, H: int, QKV, KV16, F16):
    n, m = g.n, g.m
    if QKV.size(0) < n or QKV.size(1) < 3 * D or QKV.stride(1) != 1:
        raise ValueError(f"lg bf16: QKV {tuple(QKV.shape)} must cover [{n}, >= {3 * D}] row-major")
    if KV16.dtype != torch.bfloat16 or KV16.size(0) < n or KV16.size(1) < 2 * D or KV16.stride(1) != 1:
        raise ValueError(f"lg bf16: KV16 must be bf16 [{n}, >= {2 * D}] row-major")
    if F16.dtype != torch.bfloat16 or F16.size(1) < D or F16.stride(1) != 1 or (m > 0 and F16.size(0) < m):
        raise ValueError(f"lg bf16: F16 must be bf16 [{m}, >= {D}] row-major")


def lg_fwd_bf16(g: GraphCSR, D: int, H: int, QKV, KV16, U, wbar, F16, aggV, S, sumA, mstat, den, drop_p: float,
                seed: int):
    """alignn_lg_fwd_bf16: the line-graph attention forward with bf16 K|V and edge-feature rows."""
    _check_lg_bf16(g, D, H, QKV, KV16, F16)
    if U.numel() < g.n * H * D or S.numel() < g.n * H * D or aggV.numel() < g.n * D:
        raise ValueError("lg_fwd_bf16: U and S must be [n, H, D], aggV [n, D]")
    profiling.launch(f"tconv_fwd n{g.n} m{g.m} bf16", 0.0, _lg_bf16_bytes(g.n, g.m, D, H, "fwd"),
                     lambda: check(_lib.lib().alignn_lg_fwd_bf16(
                         g.n, g.m, D, H, g.off_dst.data_ptr(), g.src_at.data_ptr(), ctypes.byref(g.schedule()),
                         QKV.data_ptr(), QKV.stride(0), KV16.data_ptr(), KV16.stride(0), U.data_ptr(), _p(wbar),
                         F16.data_ptr(), F16.stride(0), aggV.data_ptr(), S.data_ptr(), sumA.data_ptr(),
                         mstat.data_ptr(), den.data_ptr(), float(drop_p), int(seed) & (2**64 - 1), stream_ptr()),
                         "alignn_lg_fwd_bf16"))


def lg_bwd_dst_bf16(g: GraphCSR, D: int, H: int, QKV, KV16, U, Vd, wbar, F16, dout, outp, mstat, den, dq, Sz,
                    sigz, dz_e, alpha_e, drop_p: float, seed: int):
    """alignn_lg_bwd_dst_bf16: the target-side attention backward with bf16 K|V and feature rows."""
    _check_lg_bf16(g, D, H, QKV, KV16, F16)
    if (U.numel() < g.n * H * D or Vd.numel() < g.n * H * D or Sz.numel() < g.n * H * D or dq.size(0) < g.n
            or dz_e.numel() < g.m * H or alpha_e.numel() < g.m * H):
        raise ValueError("lg_bwd_dst_bf16: U, Vd, Sz [n, H, D], dq [n, >= D], dz_e/alpha_e [m, H] required")
    profiling.launch(f"tconv_bwd_dst n{g.n} m{g.m} bf16", 0.0, _lg_bf16_bytes(g.n, g.m, D, H, "bwd_dst"),
                     lambda: check(_lib.lib().alignn_lg_bwd_dst_bf16(
                         g.n, g.m, D, H, g.off_dst.data_ptr(), g.src_at.data_ptr(), ctypes.byref(g.schedule()),
                         QKV.data_ptr(), QKV.stride(0), KV16.data_ptr(), KV16.stride(0), U.data_ptr(), Vd.data_ptr(),
                         _p(wbar), F16.data_ptr(), F16.stride(0), dout.data_ptr(), outp.data_ptr(), mstat.data_ptr(),
                         den.data_ptr(), dq.data_ptr(), dq.stride(0), Sz.data_ptr(), sigz.data_ptr(),
                         dz_e.data_ptr(), alpha_e.data_ptr(), float(drop_p), int(seed) & (2**64 - 1), stream_ptr()),
                         "alignn_lg_bwd_dst_bf16"))


LGX_KIN = 11   # alignn_lg_fwd_x / _bwd_dst_x: raw angle inputs per triplet (rows of 12 floats)


def lg_x_ok(g: GraphCSR, D: int, H: int, X: Optional[torch.Tensor]) -> bool:
    """The recompute (XF) kernels' domain: D = 256, H = 4, 11 raw angle inputs in 16-byte aligned rows
    of 12 floats, a single-wave-item schedule without heavy targets."""
    return (D == 256 and H == 4 and X is not None and X.dim() == 2 and X.size(1) == LGX_KIN
            and X.stride(1) == 1 and X.stride(0) == 12 and X.data_ptr() % 16 == 0 and g.policy.wave_items
            and g.schedule().n_heavy == 0)


def _lg_x_bytes(n: int, m: int, D: int, H: int, kind: str, kv_elem: int) -> float:
    """Compulsory HBM bytes of one recompute (XF) launch: as _lg_bf16_bytes / _tconv_bytes with the
    [m, D] edge-feature rows replaced by the raw inputs (48 B per triplet) and W1 / b1."""
    xb = 48.0 * m + 4.0 * (D * LGX_KIN + D)
    if kind == "fwd":   # Q + U + CSR in (4), K|V (kv_elem), x; aggV + S + 3 stats out
        return 4.0 * (n * D + n * H * D + 2 * m + n + n * D + n * H * D + 3 * n * H) + kv_elem * 2.0 * n * D + xb
    # bwd_dst: Q,U,Vd,dout,outp,stats,CSR in; K|V; x; dQ,Sz,sigz,dz,alpha out
    return (4.0 * (n * D + 2 * n * H * D + 2 * n * D + 2 * n * H + 2 * m + n + n * D + n * H * D + n * H + 2 * m * H)
            + kv_elem * 2.0 * n * D + xb)


def _check_lg_x(g: GraphCSR, D: int, H: int, QKV, KV16, X, W1, b1):
    n, m = g.n, g.m
    if QKV.size(0) < n or QKV.size(1) < 3 * D or QKV.stride(1) != 1:
        raise ValueError(f"lg x: QKV {tuple(QKV.shape)} must cover [{n}, >= {3 * D}] row-major")
    if KV16 is not None and (KV16.dtype != torch.bfloat16 or KV16.size(0) < n or KV16.size(1) < 2 * D
                             or KV16.stride(1) != 1):
        raise ValueError(f"lg x: KV16 must be bf16 [{n}, >= {2 * D}] row-major")
    if not lg_x_ok(g, D, H, X) or (m > 0 and X.size(0) < m):
        raise ValueError(f"lg x: X must be [{m}, {LGX_KIN}] rows of 12 floats, 16-byte aligned (D = 256, H = 4, "
                         f"single-wave-item schedule)")
    if (tuple(W1.shape) != (D, LGX_KIN) or not W1.is_contiguous() or b1.numel() != D or not b1.is_contiguous()
            or W1.dtype != torch.float32 or b1.dtype != torch.float32):
        raise ValueError("lg x: W1 [256, 11] and b1 [256] contiguous fp32 required")


def lg_fwd_x(g: GraphCSR, D: int, H: int, QKV, KV16, U, wbar, X, W1, b1, aggV, S, sumA, mstat, den, drop_p: float,
             seed: int):
    """alignn_lg_fwd_x: the line-graph attention forward with the edge features recomputed from the raw
    angle inputs (f = relu(X W1^T + b1), bitwise linear_smallk; rounded to bf16 when KV16 is given —
    the bf16-storage path) instead of read from a materialised [m, D] hidden layer."""
    _check_lg_x(g, D, H, QKV, KV16, X, W1, b1)
    if U.numel() < g.n * H * D or S.numel() < g.n * H * D or aggV.numel() < g.n * D:
        raise ValueError("lg_fwd_x: U and S must be [n, H, D], aggV [n, D]")
    tag = " bf16" if KV16 is not None else ""
    profiling.launch(f"tconv_fwd n{g.n} m{g.m} x{tag}", 0.0,
                     _lg_x_bytes(g.n, g.m, D, H, "fwd", 2 if KV16 is not None else 4),
                     lambda: check(_lib.lib().alignn_lg_fwd_x(
                         g.n, g.m, D, H, g.off_dst.data_ptr(), g.src_at.data_ptr(), ctypes.byref(g.schedule()),
                         QKV.data_ptr(), QKV.stride(0), _p(KV16), 0 if KV16 is None else KV16.stride(0),
                         U.data_ptr(), _p(wbar), X.data_ptr(), X.stride(0), X.size(1), W1.data_ptr(), b1.data_ptr(),
                         aggV.data_ptr(), S.data_ptr(), sumA.data_ptr(), mstat.data_ptr(), den.data_ptr(),
                         float(drop_p), int(seed) & (2**64 - 1), stream_ptr()), "alignn_lg_fwd_x"))


def lg_bwd_dst_x(g: GraphCSR, D: int, H: int, QKV, KV16, U, Vd, wbar, X, W1, b1, dout, outp, mstat, den, dq, Sz,
                 sigz, dz_e, alpha_e, drop_p: float, seed: int):
    """alignn_lg_bwd_dst_x: the target-side attention backward with the edge features recomputed."""
    _check_lg_x(g, D, H, QKV, KV16, X, W1, b1)
    if (U.numel() < g.n * H * D or Vd.numel() < g.n * H * D or Sz.numel() < g.n * H * D or dq.size(0) < g.n
            or dz_e.numel() < g.m * H or alpha_e.numel() < g.m * H):
        raise ValueError("lg_bwd_dst_x: U, Vd, Sz [n, H, D], dq [n, >= D], dz_e/alpha_e [m, H] required")
    tag = " bf16" if KV16 is not None else ""
    profiling.launch(f"tconv_bwd_dst n{g.n} m{g.m} x{tag}", 0.0,
                     _lg_x_bytes(g.n, g.m, D, H, "bwd_dst", 2 if KV16 is not None else 4),
                     lambda: check(_lib.lib().alignn_lg_bwd_dst_x(
                         g.n, g.m, D, H, g.off_dst.data_ptr(), g.src_at.data_ptr(), ctypes.byref(g.schedule()),
                         QKV.data_ptr(), QKV.stride(0), _p(KV16), 0 if KV16 is None else KV16.stride(0),
                         U.data_ptr(), Vd.data_ptr(), _p(wbar), X.data_ptr(), X.stride(0), X.size(1), W1.data_ptr(),
                         b1.data_ptr(), dout.data_ptr(), outp.data_ptr(), mstat.data_ptr(), den.data_ptr(),
                         dq.data_ptr(), dq.stride(0), Sz.data_ptr(), sigz.data_ptr(), dz_e.data_ptr(),
                         alpha_e.data_ptr(), float(drop_p), int(seed) & (2**64 - 1), stream_ptr()),
                         "alignn_lg_bwd_dst_x"))


def cast_bf16(src: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out (bf16, round to nearest even) = src (fp32 [rows, cols], cols % 4 == 0)."""
    if out is None:
        out = torch.empty(src.shape, device=src.device, dtype=torch.bfloat16)
    if (src.dim() != 2 or src.dtype != torch.float32 or src.stride(1) != 1 or out.dtype != torch.bfloat16
            or out.stride(1) != 1 or tuple(out.shape) != tuple(src.shape)):
        raise ValueError("cast_bf16: fp32 [rows, cols] row-major source and a bf16 output of the same shape")
    check(_lib.lib().alignn_cast_bf16_f32(src.data_ptr(), src.stride(0), src.size(0), src.size(1), out.data_ptr(),
                                          out.stride(0), stream_ptr()), "alignn_cast_bf16_f32")
    return out


def tconv_bwd_src(g: GraphCSR, D: int, H: int, QKVR, dout, dz_e, alpha_e, dKV, by_source: bool = True,
                  Q16: Optional[torch.Tensor] = None, dout16: Optional[torch.Tensor] = None):
    """Source-side attention backward.  by_source: over the by-source target list
    (alignn_tconv_bwd_src_by, the default); False: the plain entry (alignn_tconv_bwd_src), same bits.
    Q16 / dout16 (bf16 storage, both or neither): the gathered target rows from bf16 copies
    (alignn_tconv_bwd_src_by_bf16; QKVR and dout are then not read)."""
    if (QKVR.size(0) < g.n or dout.numel() < g.n * D or dKV.size(0) < g.n or dKV.size(1) < 2 * D
            or dz_e.numel() < g.m * H or alpha_e.numel() < g.m * H):
        raise ValueError("tconv_bwd_src: operands do not cover the graph's n nodes / m edges")
    if (Q16 is None) != (dout16 is None):
        raise ValueError("tconv_bwd_src: Q16 and dout16 go together")
    if Q16 is not None and g.m > 0:
        for t, what in ((Q16, "Q16"), (dout16, "dout16")):
            if t.dtype != torch.bfloat16 or t.size(0) < g.n or t.size(1) < D or t.stride(1) != 1:
                raise ValueError(f"tconv_bwd_src: {what} must be bf16 [n, >= D] row-major")
        if not dout16.is_contiguous() or dout16.size(1) != D:
            raise ValueError("tconv_bwd_src: dout16 must be a contiguous [n, D] tensor")
        ds = g.dst_src()
        fn = lambda: check(_lib.lib().alignn_tconv_bwd_src_by_bf16(  # noqa: E731
            g.n, g.m, D, H, g.off_src.data_ptr(), g.pos_src.data_ptr(), ds.data_ptr(), Q16.data_ptr(),
            Q16.stride(0), dout16.data_ptr(), dz_e.data_ptr(), alpha_e.data_ptr(), dKV.data_ptr(), dKV.stride(0),
            stream_ptr()), "alignn_tconv_bwd_src_by_bf16")
        nbytes = _tconv_bytes(g.n, g.m, D, H, "bwd_src") - 4.0 * g.n * D   # Q and dout rows at 2 bytes
        profiling.launch(f"tconv_bwd_src n{g.n} m{g.m} Q16", 0.0, nbytes, fn)
        return
    if by_source and g.m > 0:
        ds = g.dst_src()
        fn = lambda: check(_lib.lib().alignn_tconv_bwd_src_by(  # noqa: E731
            g.n, g.m, D, H, g.off_src.data_ptr(), g.pos_src.data_ptr(), ds.data_ptr(), QKVR.data_ptr(),
            QKVR.stride(0), dout.data_ptr(), dz_e.data_ptr(), alpha_e.data_ptr(), dKV.data_ptr(), dKV.stride(0),
            stream_ptr()), "alignn_tconv_bwd_src_by")
    else:
        fn = lambda: check(_lib.lib().alignn_tconv_bwd_src(  # noqa: E731
            g.n, g.m, D, H, g.off_src.data_ptr(), g.pos_src.data_ptr(), g.dst_at.data_ptr(), QKVR.data_ptr(),
            QKVR.stride(0), dout.data_ptr(), dz_e.data_ptr(), alpha_e.data_ptr(), dKV.data_ptr(), dKV.stride(0),
            stream_ptr()), "alignn_tconv_bwd_src")
    profiling.launch(f"tconv_bwd_src n{g.n} m{g.m}", 0.0, _tconv_bytes(g.n, g.m, D, H, "bwd_src"), fn)


# ------------------------------------------------------------------------------------------------
# Row ops
# ------------------------------------------------------------------------------------------------
def _check_outp_rows(outp, outp_rows, n):
    if outp_rows is None:
        if outp.size(0) != n:
            raise ValueError(f"gate_ln: outp has {outp.size(0)} rows, expected {n}")
        return None
    if outp_rows.dtype != torch.int32 or outp_rows.numel() != n or not outp_rows.is_contiguous():
        raise ValueError("gate_ln: outp_rows must be contiguous int32 with one entry per row")
    return outp_rows.data_ptr()


def gate_ln_fwd(outp, R, wbeta, X, ln_w, ln_b, Xnew, beta, mu, rstd, drop_p, seed, outp_rows=None, Xnew16=None,
                Xa_out=None):
    """outp_rows (int32 [n], -1 = zero row): o of row r is outp[outp_rows[r]] (compacted conv output).
    R may be bf16 (the skip projection's bf16 output); Xnew16 (bf16 [n, D], optional) receives a bf16
    copy of the new state (alignn_gate_ln_fwd_ex).  Xa_out (fp32 contiguous [outp rows, D], needs
    outp_rows): row r of the new state also goes to Xa_out[outp_rows[r]] where that is >= 0 — the
    next line block's active-row gather (alignn_gate_ln_fwd_ex2)."""
    n, D = X.shape
    rp = _check_outp_rows(outp, outp_rows, n)
    if Xa_out is not None:
        _require(Xa_out, "gate_ln_fwd Xa_out")
        if outp_rows is None or tuple(Xa_out.shape) != tuple(outp.shape) or not Xa_out.is_contiguous():
            raise ValueError("gate_ln_fwd: Xa_out must be a contiguous tensor of outp's shape (with outp_rows)")
        if Xnew16 is not None and (Xnew16.dtype != torch.bfloat16 or tuple(Xnew16.shape) != (n, D)
                                   or Xnew16.stride(1) != 1):
            raise ValueError("gate_ln_fwd: Xnew16 must be a bf16 [n, D] row-major tensor")
        check(_lib.lib().alignn_gate_ln_fwd_ex2(n, D, outp.data_ptr(), rp, R.data_ptr(), R.stride(0),
                                                int(R.dtype == torch.bfloat16), wbeta.data_ptr(), X.data_ptr(),
                                                X.stride(0), ln_w.data_ptr(), ln_b.data_ptr(), Xnew.data_ptr(),
                                                Xnew.stride(0), _p(Xnew16), 0 if Xnew16 is None else Xnew16.stride(0),
                                                Xa_out.data_ptr(), beta.data_ptr(), mu.data_ptr(), rstd.data_ptr(),
                                                float(drop_p), int(seed) & (2**64 - 1), stream_ptr()),
              "alignn_gate_ln_fwd_ex2")
        return
    if R.dtype == torch.bfloat16 or Xnew16 is not None:
        if Xnew16 is not None and (Xnew16.dtype != torch.bfloat16 or tuple(Xnew16.shape) != (n, D)
                                   or Xnew16.stride(1) != 1):
            raise ValueError("gate_ln_fwd: Xnew16 must be a bf16 [n, D] row-major tensor")
        check(_lib.lib().alignn_gate_ln_fwd_ex(n, D, outp.data_ptr(), rp, R.data_ptr(), R.stride(0),
                                               int(R.dtype == torch.bfloat16), wbeta.data_ptr(), X.data_ptr(),
                                               X.stride(0), ln_w.data_ptr(), ln_b.data_ptr(), Xnew.data_ptr(),
                                               Xnew.stride(0), _p(Xnew16), 0 if Xnew16 is None else Xnew16.stride(0),
                                               beta.data_ptr(), mu.data_ptr(), rstd.data_ptr(), float(drop_p),
                                               int(seed) & (2**64 - 1), stream_ptr()), "alignn_gate_ln_fwd_ex")
        return
    check(_lib.lib().alignn_gate_ln_fwd_rows(n, D, outp.data_ptr(), rp, R.data_ptr(), R.stride(0), wbeta.data_ptr(),
                                             X.data_ptr(), X.stride(0), ln_w.data_ptr(), ln_b.data_ptr(),
                                             Xnew.data_ptr(), Xnew.stride(0), beta.data_ptr(), mu.data_ptr(),
                                             rstd.data_ptr(), float(drop_p), int(seed) & (2**64 - 1), stream_ptr()),
          "alignn_gate_ln_fwd")


def gate_ln_bwd(dXnew, outp, R, wbeta, ln_w, ln_b, beta, mu, rstd, dout, dR, d_wbeta, d_ln_w, d_ln_b, drop_p, seed,
                outp_rows=None, reduce_stream: Optional[torch.cuda.Stream] = None,
                dX_add: Optional[torch.Tensor] = None, dX_zero: bool = False):
    """outp_rows: as in gate_ln_fwd; dout then has outp's (compacted) rows and only those are written.
    reduce_stream: run the parameter-gradient reduction (d_wbeta, d_ln_w, d_ln_b) there, after the
    row kernel, off the current stream (nothing on it reads those gradients).
    dX_add: [n, D] contiguous addend of the incoming gradient; dXnew += dX_add is written back
    (alignn_gate_ln_bwd_partials_add).  dX_zero: dXnew holds nothing yet (read as zero, not loaded;
    needs dX_add): the incoming gradient is dX_add, written to dXnew."""
    n, D = R.shape
    rp = _check_outp_rows(outp, outp_rows, n)
    if dout.shape != outp.shape:
        raise ValueError("gate_ln_bwd: dout must have outp's shape")
    wsize = int(_lib.lib().alignn_gate_ln_bwd_workspace(int(n), D))
    x2bf = dX_add is not None and dX_add.dtype == torch.bfloat16
    if dX_zero and dX_add is None:
        raise ValueError("gate_ln_bwd: dX_zero needs dX_add")
    if R.dtype == torch.bfloat16 or dR.dtype == torch.bfloat16 or x2bf or dX_zero:
        # bf16 storage: R read / dR written / dX_add read in bf16 (alignn_gate_ln_bwd_partials_ex + _reduce)
        if dX_add is not None:
            _require(dX_add, "gate_ln_bwd dX_add", dX_add.dtype if x2bf else torch.float32)
            if tuple(dX_add.shape) != (n, D) or not dX_add.is_contiguous():
                raise ValueError("gate_ln_bwd: dX_add must be a contiguous [n, D] tensor")
        red = reduce_stream if reduce_stream is not None else torch.cuda.current_stream(outp.device)
        ws = (current().fresh("gate_ln_red", wsize, outp.device) if reduce_stream is not None
              else WS.get("gate_ln", wsize, outp.device))
        check(_lib.lib().alignn_gate_ln_bwd_partials_ex(n, D, dXnew.data_ptr(), dXnew.stride(0), _p(dX_add),
                                                        outp.data_ptr(), rp, R.data_ptr(), R.stride(0),
                                                        int(R.dtype == torch.bfloat16) | (2 if x2bf else 0)
                                                        | (4 if dX_zero else 0),
                                                        wbeta.data_ptr(),
                                                        ln_w.data_ptr(), ln_b.data_ptr(), beta.data_ptr(),
                                                        mu.data_ptr(), rstd.data_ptr(), dout.data_ptr(), dR.data_ptr(),
                                                        dR.stride(0), int(dR.dtype == torch.bfloat16), ws.data_ptr(),
                                                        float(drop_p), int(seed) & (2**64 - 1), stream_ptr()),
              "alignn_gate_ln_bwd_partials_ex")
        if reduce_stream is not None:
            stream_wait(reduce_stream, torch.cuda.current_stream(outp.device))
            ws.record_stream(reduce_stream)
        check(_lib.lib().alignn_gate_ln_bwd_reduce(n, D, ws.data_ptr(), d_wbeta.data_ptr(), d_ln_w.data_ptr(),
                                                   d_ln_b.data_ptr(), red.cuda_stream), "alignn_gate_ln_bwd_reduce")
        return
    if dX_add is not None:
        _require(dX_add, "gate_ln_bwd dX_add")
        if tuple(dX_add.shape) != (n, D) or not dX_add.is_contiguous():
            raise ValueError("gate_ln_bwd: dX_add must be a contiguous [n, D] tensor")
        red = reduce_stream if reduce_stream is not None else torch.cuda.current_stream(outp.device)
        ws = (current().fresh("gate_ln_red", wsize, outp.device) if reduce_stream is not None
              else WS.get("gate_ln", wsize, outp.device))
        check(_lib.lib().alignn_gate_ln_bwd_partials_add(n, D, dXnew.data_ptr(), dXnew.stride(0), dX_add.data_ptr(),
                                                         outp.data_ptr(), rp, R.data_ptr(), R.stride(0),
                                                         wbeta.data_ptr(), ln_w.data_ptr(), ln_b.data_ptr(),
                                                         beta.data_ptr(), mu.data_ptr(), rstd.data_ptr(),
                                                         dout.data_ptr(), dR.data_ptr(), dR.stride(0), ws.data_ptr(),
                                                         float(drop_p), int(seed) & (2**64 - 1), stream_ptr()),
              "alignn_gate_ln_bwd_partials_add")
        if reduce_stream is not None:
            stream_wait(reduce_stream, torch.cuda.current_stream(outp.device))
            ws.record_stream(reduce_stream)
        check(_lib.lib().alignn_gate_ln_bwd_reduce(n, D, ws.data_ptr(), d_wbeta.data_ptr(), d_ln_w.data_ptr(),
                                                   d_ln_b.data_ptr(), red.cuda_stream),
              "alignn_gate_ln_bwd_reduce")
        return
    if reduce_stream is not None:
        ws = current().fresh("gate_ln_red", wsize, outp.device)   # its own buffer: read later on reduce_stream
        check(_lib.lib().alignn_gate_ln_bwd_partials(n, D, dXnew.data_ptr(), dXnew.stride(0), outp.data_ptr(), rp,
                                                     R.data_ptr(), R.stride(0), wbeta.data_ptr(), ln_w.data_ptr(),
                                                     ln_b.data_ptr(), beta.data_ptr(), mu.data_ptr(), rstd.data_ptr(),
                                                     dout.data_ptr(), dR.data_ptr(), dR.stride(0), ws.data_ptr(),
                                                     float(drop_p), int(seed) & (2**64 - 1), stream_ptr()),
              "alignn_gate_ln_bwd_partials")
        stream_wait(reduce_stream, torch.cuda.current_stream(outp.device))
        ws.record_stream(reduce_stream)
        check(_lib.lib().alignn_gate_ln_bwd_reduce(n, D, ws.data_ptr(), d_wbeta.data_ptr(), d_ln_w.data_ptr(),
                                                   d_ln_b.data_ptr(), reduce_stream.cuda_stream),
              "alignn_gate_ln_bwd_reduce")
        return
    ws = WS.get("gate_ln", wsize, outp.device)
    check(_lib.lib().alignn_gate_ln_bwd_rows(n, D, dXnew.data_ptr(), dXnew.stride(0), outp.data_ptr(), rp,
                                             R.data_ptr(), R.stride(0), wbeta.data_ptr(), ln_w.data_ptr(),
                                             ln_b.data_ptr(), beta.data_ptr(), mu.data_ptr(), rstd.data_ptr(),
                                             dout.data_ptr(), dR.data_ptr(), dR.stride(0), d_wbeta.data_ptr(),
                                             d_ln_w.data_ptr(), d_ln_b.data_ptr(), ws.data_ptr(), float(drop_p),
                                             int(seed) & (2**64 - 1), stream_ptr()), "alignn_gate_ln_bwd")


def readout_feats_fwd(h, ptr, global_x, gdim, sg, sgdim, feats, drop_p, seed):
    B = ptr.numel() - 1
    D = h.size(1)
    check(_lib.lib().alignn_readout_feats_fwd(B, D, h.data_ptr(), ptr.data_ptr(), global_x.data_ptr(), gdim,
                                              sg.data_ptr(), sgdim, feats.data_ptr(), float(drop_p),
                                              int(seed) & (2**64 - 1), stream_ptr()), "alignn_readout_feats_fwd")


def readout_pool_bwd(dfeats, ptr, batch, dh, accumulate, drop_p, seed):
    B = ptr.numel() - 1
    N, D = dh.shape
    check(_lib.lib().alignn_readout_pool_bwd(B, N, D, dfeats.data_ptr(), dfeats.stride(0), ptr.data_ptr(),
                                             batch.data_ptr(), dh.data_ptr(), int(accumulate), float(drop_p),
                                             int(seed) & (2**64 - 1), stream_ptr()), "alignn_readout_pool_bwd")


def dropout(x, y, relu_ref=None, drop_p=0.0, seed=0):
    rows, cols = x.shape
    check(_lib.lib().alignn_dropout_f32(rows, cols, x.data_ptr(), x.stride(0), y.data_ptr(), y.stride(0),
                                        _p(relu_ref), 0 if relu_ref is None else relu_ref.stride(0), float(drop_p),
                                        int(seed) & (2**64 - 1), stream_ptr()), "alignn_dropout_f32")
    return y


def hetero_nll(heads, y, log_means, log_stds, floor, l2, loss, dheads, weights: Optional[torch.Tensor] = None,
               amp: bool = False):
    """weights: per-graph KNN sample weights [B] (train.py:660-674) or None.  amp: the loss as the
    reference's CUDA step computes it under autocast(bfloat16) on bf16 heads (alignn_hetero_nll_amp)."""
    B = heads.size(0)
    T = heads.size(1) // 2
    if weights is not None and (weights.numel() != B or weights.dtype != torch.float32 or not weights.is_contiguous()):
        raise ValueError("hetero_nll: weights must be a contiguous float32 [B] tensor")
    fn = _lib.lib().alignn_hetero_nll_amp if amp else _lib.lib().alignn_hetero_nll
    check(fn(B, T, heads.data_ptr(), heads.stride(0), y.data_ptr(), _p(weights), log_means.data_ptr(),
             log_stds.data_ptr(), float(floor), float(l2), loss.data_ptr(), dheads.data_ptr(), dheads.stride(0),
             stream_ptr()), "alignn_hetero_nll_amp" if amp else "alignn_hetero_nll")


def add_noise(x: torch.Tensor, std: float, seed: int):
    check(_lib.lib().alignn_add_noise_f32(x.numel(), x.data_ptr(), float(std), int(seed) & (2**64 - 1),
                                          stream_ptr()), "alignn_add_noise_f32")


def noisy_copies(x1: torch.Tensor, seed1: int, x2: torch.Tensor, seed2: int, std: float):
    """(x1 + std * N(0, 1), x2 + std * N(0, 1)) as new contiguous fp32 tensors in one launch: the same
    values as clone() + add_noise(seed_k) of each (alignn_noisy_copy2_f32)."""
    _require(x1, "x1")
    _require(x2, "x2")
    x1, x2 = x1.contiguous(), x2.contiguous()
    y1, y2 = torch.empty_like(x1), torch.empty_like(x2)
    if std == 0.0:
        copy_many([(y1, x1), (y2, x2)])
        return y1, y2
    check(_lib.lib().alignn_noisy_copy2_f32(x1.numel(), x1.data_ptr(), y1.data_ptr(), int(seed1) & (2**64 - 1),
                                            x2.numel(), x2.data_ptr(), y2.data_ptr(), int(seed2) & (2**64 - 1),
                                            float(std), stream_ptr()), "alignn_noisy_copy2_f32")
    return y1, y2


# ------------------------------------------------------------------------------------------------
# Optimizer (clip_grad_norm_ + AdamW over the flat buffers)
# ------------------------------------------------------------------------------------------------
def grad_norm(g: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    _require(g, "g")
    ws = WS.get("gnorm", 1024, g.device)
    check(_lib.lib().alignn_grad_norm_f32(g.data_ptr(), g.numel(), out.data_ptr(), ws.data_ptr(), stream_ptr()),
          "alignn_grad_norm_f32")
    return out


def _check_scaler(scaler: torch.Tensor) -> None:
    _require(scaler, "scaler")
    if scaler.numel() != 4 or not scaler.is_contiguous():
        raise ValueError("scaler must be a contiguous float32 device tensor [scale, growth_tracker, found_inf, skipped]")


def grad_norm_amp(g: torch.Tensor, out: torch.Tensor, scaler: torch.Tensor) -> torch.Tensor:
    """grad_norm plus GradScaler.unscale_'s found-inf flag in scaler[2] (alignn_grad_norm_amp_f32)."""
    _require(g, "g")
    _check_scaler(scaler)
    ws = WS.get("gnorm", 2048, g.device)
    check(_lib.lib().alignn_grad_norm_amp_f32(g.data_ptr(), g.numel(), out.data_ptr(), scaler.data_ptr(), ws.data_ptr(),
                                              stream_ptr()), "alignn_grad_norm_amp_f32")
    return out


def adamw_step(p: torch.Tensor, g: torch.Tensor, m: torch.Tensor, v: torch.Tensor, split: int, lr0: float,
               lr1: float, weight_decay: float, betas=(0.9, 0.999), eps: float = 1e-8,
               norm: Optional[torch.Tensor] = None, max_norm: float = 5.0, step: torch.Tensor = None,
               lr_dev: Optional[torch.Tensor] = None, scaler: Optional[torch.Tensor] = None,
               growth_interval: int = 2000) -> None:
    """lr_dev: device float64 [2] = (lr0, lr1) read by the kernel when it runs (lr0/lr1 ignored), so a
    recorded plan follows learning-rate changes (alignn_adamw_f32_dev).  scaler (with lr_dev): the
    GradScaler state of grad_norm_amp — a flagged step is skipped and the scale backs off
    (alignn_adamw_amp_f32_dev)."""
    for t, n in ((p, "p"), (g, "g"), (m, "m"), (v, "v")):
        _require(t, n)
        if not t.is_contiguous() or t.numel() != p.numel():
            raise ValueError(f"adamw_step: {n} must be contiguous with {p.numel()} elements")
    if scaler is not None:
        _check_scaler(scaler)
        if lr_dev is None:
            raise ValueError("adamw_step: the GradScaler form reads device learning rates (lr_dev)")
        _require(lr_dev, "lr_dev", torch.float64)
        check(_lib.lib().alignn_adamw_amp_f32_dev(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(),
                                                  int(split), lr_dev.data_ptr(), float(weight_decay), float(betas[0]),
                                                  float(betas[1]), float(eps), _p(norm), float(max_norm),
                                                  step.data_ptr(), scaler.data_ptr(), int(growth_interval),
                                                  stream_ptr()), "alignn_adamw_amp_f32_dev")
        return
    if lr_dev is not None:
        _require(lr_dev, "lr_dev", torch.float64)
        if lr_dev.numel() != 2 or not lr_dev.is_contiguous():
            raise ValueError("adamw_step: lr_dev must be a contiguous float64 tensor of 2 elements")
        check(_lib.lib().alignn_adamw_f32_dev(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(),
                                              int(split), lr_dev.data_ptr(), float(weight_decay), float(betas[0]),
                                              float(betas[1]), float(eps), _p(norm), float(max_norm), step.data_ptr(),
                                              stream_ptr()), "alignn_adamw_f32_dev")
        return
    check(_lib.lib().alignn_adamw_f32(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), int(split),
                                      float(lr0), float(lr1), float(weight_decay), float(betas[0]), float(betas[1]),
                                      float(eps), _p(norm), float(max_norm), step.data_ptr(), stream_ptr()),
          "alignn_adamw_f32")
