"""Round-6 checks.

* Host reads right after a replayed plan: the step's cross-stream edges carry no
  system-scope fence, except the final joins into the caller's stream (plan.hip alignn_plan_end).  The
  loss read with .item() and the gradients / parameters copied to the host straight after each replay —
  no explicit synchronize in between — equal the eager step's bit for bit, at B = 4 and at the bench's
  B = 32 (whose step joins the side and aux streams).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(B):
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    torch.manual_seed(0)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
    return A.FusedTrainer(model), mp_like_batch(B).to(DEV)


@pytest.mark.parametrize("B", [4, 32])
def test_replayed_step_host_reads_equal_eager(B):
    from alignn_mi355x import ops
    tr1, b1 = _setup(B)
    tr2, b2 = _setup(B)
    tr2.capture(b2)
    try:
        for s in (21, 22, 23):
            tr1.use_step_seed(tr2._seed_dev)
            tr2._seed_dev.fill_(s)
            tr1.forward_backward(b1, 0)
            tr1._clip_and_update()
            l1, g1, p1 = tr1.loss.item(), tr1.st.grad.cpu(), tr1.st.flat.cpu()
            l2 = tr2.step(b2, seed=s).item()        # D2H straight after the replay's last join
            g2, p2 = tr2.st.grad.cpu(), tr2.st.flat.cpu()
            assert l1 == l2, s
            assert torch.equal(g1, g2), s
            assert torch.equal(p1, p2), s
    finally:
        ops.set_step_seed(None)


@pytest.mark.parametrize("add_bf16", [False, True])
def test_gate_bwd_dx_zero_equals_zero_filled_plus_add(add_bf16):
    """the gate backward's zero-free incoming gradient (dX_zero: the last line block,
    whose only consumer is the atom block beside it, engine._backward_layers de_fresh) against a
    zero-filled dX with the same addend — the per-row outputs bitwise, the parameter gradients to fp32
    rounding, for an fp32 and a bf16 addend (the atom blocks' edge-feature gradient in bf16 storage)."""
    from alignn_mi355x import ops
    ops.set_step_seed(None)
    n, D = 2000, 256
    g = torch.Generator(device="cpu").manual_seed(5)
    r = lambda *s: torch.randn(*s, generator=g).to(DEV)  # noqa: E731
    R16, X, outp = r(n, D).bfloat16(), r(n, D), r(n, D)
    wbeta, lnw, lnb = 0.1 * r(3 * D), 1 + 0.1 * r(D), 0.1 * r(D)
    add = r(n, D)
    add = add.bfloat16() if add_bf16 else add
    Xn = torch.empty(n, D, device=DEV)
    beta, mu, rstd = (torch.empty(n, device=DEV) for _ in range(3))
    ops.gate_ln_fwd(outp, R16, wbeta, X, lnw, lnb, Xn, beta, mu, rstd, 0.15, 77)
    res = []
    for zero in (False, True):
        dXn = torch.full((n, D), float("nan"), device=DEV) if zero else torch.zeros(n, D, device=DEV)
        dout, dR = torch.empty_like(outp), torch.empty(n, D, device=DEV, dtype=torch.bfloat16)
        grads = [torch.zeros(3 * D, device=DEV), torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)]
        ops.gate_ln_bwd(dXn, outp, R16, wbeta, lnw, lnb, beta, mu, rstd, dout, dR, *grads, 0.15, 77, dX_add=add,
                        dX_zero=zero)
        res.append((dXn, dout, dR, *grads))
    torch.cuda.synchronize()
    a, b = res
    for i in (0, 1, 2):   # per-row outputs (dX, dout, dR): bitwise
        assert torch.equal(a[i], b[i]), i
    for i in (3, 4, 5):   # parameter gradients (fixed-order sums over rows): the two row-kernel variants may
        # contract the per-row partials' fmas differently (as tests/test_gpu_x_bf16_io.py): fp32 rounding
        err = float((a[i] - b[i]).abs().max() / b[i].abs().max())
        assert err < 1e-6, (i, err)


@pytest.mark.parametrize("cols,ld", [(256, 256), (260, 264), (30, 30), (8, 12)])
def test_row_moves_vector_and_element_paths(cols, ld):
    """graph.hip gather / scatter rows: the wave-per-row 16-byte path (cols and leading dimensions
    multiples of 4: 256, and 260 = more float4s per row than lanes) and the element loop (30; 8 with
    an odd start column below) — each a plain copy, so bitwise against torch indexing, with and
    without accumulation."""
    from alignn_mi355x import ops
    torch.manual_seed(11)
    n, na = 3000, 777
    rows = torch.randperm(n)[:na].to(torch.int32).to(DEV)
    big = torch.randn(n, ld, device=DEV)
    src = big[:, :cols] if (cols, ld) != (8, 12) else big[:, 1:9]
    g = ops.gather_rows(src, rows)
    assert torch.equal(g, src[rows.long()])
    vals = torch.randn(na, ld, device=DEV)[:, :cols]
    out0 = torch.randn(n, ld, device=DEV)
    out = out0.clone()
    ops.scatter_rows(vals, rows, out[:, :cols])
    ref = out0.clone()
    ref[rows.long(), :cols] = vals
    assert torch.equal(out, ref)
    out = out0.clone()
    ops.scatter_rows(vals, rows, out[:, :cols], accumulate=True)
    ref = out0.clone()
    ref[rows.long(), :cols] += vals
    assert torch.equal(out, ref)
