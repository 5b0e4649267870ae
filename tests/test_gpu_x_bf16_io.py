"""bf16 storage kernels (config C3, the reference's autocast dtypes — Linear outputs and their
gradients in bf16, train.py:632-636): GEMMs reading bf16 operands or writing a bf16 output, the
bf16 column sum, and the gate/LayerNorm kernels reading R / writing dR and the state's bf16 copy.
Each is checked BIT FOR BIT against the fp32-storage kernel on the bf16-rounded values: widening
bf16 -> fp32 is exact and the bf16 matrix cores round their fp32 inputs to the same bf16 values, so
only the output rounding (RNE of the same fp32 value) may differ — and that is reproduced exactly."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rand(*shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(*shape, generator=g).to(DEV)


# (M, N, K): the streaming kernel's shape (M >= 4096, N % 256, K = 256) and tiled shapes (small M,
# ragged edges, long-K weight gradients)
@pytest.mark.parametrize("M,N,K", [(23040, 256, 256), (5000, 256, 256), (2880, 256, 256), (999, 130, 72)])
@pytest.mark.parametrize("which", ["A", "C", "AC"])
def test_gemm_bf16_operand_and_output_bitwise(M, N, K, which):
    from alignn_mi355x import ops
    A32 = _rand(M, K, seed=1)
    W = _rand(N, K, seed=2)
    bias = _rand(N, seed=3)
    A16 = A32.bfloat16()
    Aop = A16 if "A" in which else A16.float()
    with ops.gemm_precision("bf16"):
        ref = torch.empty(M, N, device=DEV)
        ops.gemm(A16.float(), W.t(), ref, bias=bias)
        if "C" in which:
            out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ops.gemm(Aop, W.t(), out, bias=bias)
            torch.cuda.synchronize()
            assert torch.equal(out, ref.bfloat16())
        else:
            out = torch.empty(M, N, device=DEV)
            ops.gemm(Aop, W.t(), out, bias=bias)
            torch.cuda.synchronize()
            assert torch.equal(out, ref)


@pytest.mark.parametrize("M,K", [(23040, 256), (2880, 256)])
def test_gemm_bf16_A_with_beta_accumulates_in_fp32(M, K):
    """The skip projection's dX product: dX += dR16 W (C fp32, beta = 1)."""
    from alignn_mi355x import ops
    dR16 = _rand(M, K, seed=4).bfloat16()
    W = _rand(K, 256, seed=5)
    C0 = _rand(M, 256, seed=6)
    with ops.gemm_precision("bf16"):
        a, b = C0.clone(), C0.clone()
        ops.gemm(dR16, W, a, beta=1.0)
        ops.gemm(dR16.float(), W, b, beta=1.0)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


@pytest.mark.parametrize("rows", [184320, 23040, 2880])
def test_weight_gradient_with_bf16_operands_bitwise(rows):
    """dW = dR16^T X16 (both bf16, long K = rows: split-K plans) and its bias colsum."""
    from alignn_mi355x import ops
    dR16 = _rand(rows, 256, seed=7).bfloat16()
    X16 = _rand(rows, 256, seed=8).bfloat16()
    with ops.gemm_precision("bf16"):
        w1 = torch.empty(256, 256, device=DEV)
        w2 = torch.empty(256, 256, device=DEV)
        ops.gemm(dR16.t(), X16, w1)
        ops.gemm(dR16.float().t(), X16.float(), w2)
    b1 = torch.empty(256, device=DEV)
    b2 = torch.empty(256, device=DEV)
    ops.colsum(dR16, b1)
    ops.colsum(dR16.float(), b2)
    torch.cuda.synchronize()
    assert torch.equal(w1, w2)
    assert torch.equal(b1, b2)


def test_bf16_gemm_output_refuses_beta():
    from alignn_mi355x import ops
    from alignn_mi355x._lib import AlignnHipError
    with ops.gemm_precision("bf16"):
        C = torch.zeros(64, 64, device=DEV, dtype=torch.bfloat16)
        with pytest.raises(AlignnHipError):
            ops.gemm(_rand(64, 64), _rand(64, 64), C, beta=1.0)
    with pytest.raises(ValueError):   # bf16 operands need bf16 arithmetic
        ops.gemm(_rand(64, 64).bfloat16(), _rand(64, 64), torch.zeros(64, 64, device=DEV))


@pytest.mark.parametrize("compact", [False, True])
def test_gate_ln_bf16_io_bitwise(compact):
    from alignn_mi355x import ops
    ops.set_step_seed(None)   # host seeds only: the dropout masks must not read a step seed another test left
    n, D = 3000, 256
    R16 = _rand(n, D, seed=9).bfloat16()
    X = _rand(n, D, seed=10)
    wbeta = _rand(3 * D, seed=11) * 0.1
    lnw = 1 + 0.1 * _rand(D, seed=12)
    lnb = 0.1 * _rand(D, seed=13)
    if compact:
        na = 700
        outp = _rand(na, D, seed=14)
        rows_map = torch.full((n,), -1, dtype=torch.int32, device=DEV)
        idx = torch.randperm(n, generator=torch.Generator().manual_seed(15))[:na].to(DEV)
        rows_map[idx] = torch.arange(na, dtype=torch.int32, device=DEV)
    else:
        outp, rows_map = _rand(n, D, seed=14), None
    res = []
    for r in (R16, R16.float()):
        Xn = torch.empty(n, D, device=DEV)
        X16 = torch.empty(n, D, device=DEV, dtype=torch.bfloat16)
        beta, mu, rstd = (torch.empty(n, device=DEV) for _ in range(3))
        ops.gate_ln_fwd(outp, r, wbeta, X, lnw, lnb, Xn, beta, mu, rstd, 0.15, 77, outp_rows=rows_map, Xnew16=X16)
        dXn = _rand(n, D, seed=16)
        dout = torch.empty_like(outp)
        dR = torch.empty(n, D, device=DEV, dtype=r.dtype)
        g = [torch.zeros(3 * D, device=DEV), torch.zeros(D, device=DEV), torch.zeros(D, device=DEV)]
        ops.gate_ln_bwd(dXn, outp, r, wbeta, lnw, lnb, beta, mu, rstd, dout, dR, *g, 0.15, 77, outp_rows=rows_map)
        res.append((Xn, X16, beta, mu, rstd, dout, dR, *g))
    torch.cuda.synchronize()
    a, b = res
    assert torch.equal(a[1], a[0].bfloat16())           # the state's bf16 copy is RNE of the fp32 state
    for i in (0, 1, 2, 3, 4, 5):   # per-row outputs: bitwise
        assert torch.equal(a[i], b[i]), i
    for i in (7, 8, 9):            # parameter gradients (fixed-order sums over rows): the two variants of the
        # row kernel may contract the per-row partials' fmas differently; within fp32 rounding
        err = float((a[i] - b[i]).abs().max() / b[i].abs().max())
        assert err < 1e-6, (i, err)
    assert a[6].dtype == torch.bfloat16 and torch.equal(a[6], b[6].bfloat16())   # dR = RNE(fp32 dR)
