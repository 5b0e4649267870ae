"""Execution contexts (ops.ExecContext): workspaces are per engine and frozen while a launch plan is
being recorded, the default (shared) context cannot be recorded, and ``fresh`` hands out distinct
buffers within one pass.  Host logic only (CPU tensors stand in for device buffers)."""
import pytest
import torch


def test_workspace_reuse_and_growth():
    from alignn_mi355x import ops
    ctx = ops.ExecContext("t")
    a = ctx.get("gemm", 100, "cpu")
    b = ctx.get("gemm", 50, "cpu")
    assert a.data_ptr() == b.data_ptr()          # reused while large enough
    c = ctx.get("gemm", 200, "cpu")
    assert c.numel() >= 200 and ctx.get("gemm", 10, "cpu").data_ptr() == c.data_ptr()
    assert ctx.get("colsum", 10, "cpu").data_ptr() != c.data_ptr()   # per purpose


def test_workspace_frozen_while_recording():
    from alignn_mi355x import ops
    ctx = ops.ExecContext("t")
    a = ctx.get("gemm", 100, "cpu")
    with ops.recording():
        assert ctx.get("gemm", 100, "cpu").data_ptr() == a.data_ptr()  # fits: the same buffer
        with pytest.raises(RuntimeError, match="would grow"):
            ctx.get("gemm", 101, "cpu")
        with pytest.raises(RuntimeError, match="would grow"):
            ctx.get("new-purpose", 1, "cpu")
        with pytest.raises(RuntimeError, match="engine-owned"):
            ops.current().get("gemm", 1, "cpu")   # the shared default context
    assert ctx.get("gemm", 101, "cpu").numel() >= 101   # grows again outside a recording


def test_fresh_buffers_distinct_per_pass():
    from alignn_mi355x import ops
    ctx = ops.ExecContext("t")
    bufs = [ctx.fresh("red", 64, "cpu") for _ in range(3)]
    assert len({b.data_ptr() for b in bufs}) == 3
    ctx.new_pass()
    again = [ctx.fresh("red", 64, "cpu") for _ in range(3)]
    assert [b.data_ptr() for b in again] == [b.data_ptr() for b in bufs]   # same set next pass
    with ops.recording():
        ctx.new_pass()
        assert ctx.fresh("red", 64, "cpu").data_ptr() == bufs[0].data_ptr()
        with pytest.raises(RuntimeError):
            [ctx.fresh("red", 64, "cpu") for _ in range(3)]   # a 4th buffer would be new


def test_using_is_nested_and_thread_local():
    import threading
    from alignn_mi355x import ops
    c1, c2 = ops.ExecContext("a"), ops.ExecContext("b")
    seen = {}
    with ops.using(c1):
        assert ops.current() is c1
        with ops.using(c2):
            assert ops.current() is c2

            def other():
                seen["t"] = ops.current()
            th = threading.Thread(target=other)
            th.start()
            th.join()
        assert ops.current() is c1
    assert seen["t"] is not c1 and seen["t"] is not c2
    assert not ops.current().owned


def test_frozen_context_never_replaces_a_plan_buffer():
    """While a plan holds the buffers (freeze), an eager launch that needs more gets a separate
    buffer; the plan's buffer keeps its address, and after thaw the larger one takes over."""
    from alignn_mi355x import ops
    ctx = ops.ExecContext("t")
    a = ctx.get("gemm", 100, "cpu")
    ctx.freeze()
    big = ctx.get("gemm", 500, "cpu")
    assert big.data_ptr() != a.data_ptr() and big.numel() >= 500
    assert ctx.buf[next(k for k in ctx.buf if k[0] == "gemm")].data_ptr() == a.data_ptr()
    assert ctx.get("gemm", 50, "cpu").data_ptr() == a.data_ptr()      # fits: the plan's buffer
    assert ctx.get("gemm", 400, "cpu").data_ptr() == big.data_ptr()   # the eager overflow is reused
    assert a.data_ptr() in {t.data_ptr() for t in ctx.tensors()}
    ctx.thaw()
    assert ctx.get("gemm", 500, "cpu").data_ptr() == big.data_ptr()


def test_default_context_keys_buffers_by_stream():
    """The shared default context keys its buffers by the stream itself (a loader stream and the
    main stream never share a scratch buffer); an engine context keys the current stream as 'main'."""
    from alignn_mi355x import ops
    d = ops.ExecContext("default", owned=False)
    assert d._role("cpu") == "main"
    e = ops.ExecContext("engine")
    assert e._role("cpu") == "main"
