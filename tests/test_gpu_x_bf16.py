"""bf16 GEMM arithmetic (ALIGNN_GEMM_BF16; SURVEY §8d config C3 — the reference's CUDA autocast
GEMMs, train.py:632-636): inputs rounded to bf16 (RNE) into v_mfma_f32_32x32x16_bf16, fp32
accumulation and storage.  The exact reference for that arithmetic is an fp64 product of the
bf16-rounded operands (bf16 x bf16 products are exact in fp32, so only the fp32 summation order
differs): tolerance 5e-6 relative to the largest output.  Engine level: a bf16 training step against
the fp32 one (loss within 2e-2 relative, gradient cosine > 0.999).  Sorts after the core suites."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


def _rb(x):
    return x.bfloat16().double()


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 17, 20])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
def test_gemm_bf16_layouts_and_tiles(tile, layout):
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(tile * 5 + len(layout) + ord(layout[0]))
    M, N, K = 300, 257, 1000
    A = torch.randn(M, K, generator=g).to(DEV)
    B = torch.randn(K, N, generator=g).to(DEV)
    Av = A if layout[0] == "n" else A.t().contiguous().t()
    Bv = B if layout[1] == "n" else B.t().contiguous().t()
    ref = _rb(A) @ _rb(B)
    for split in (1, 3):
        C = torch.empty(M, N, device=DEV)
        ops.gemm(Av, Bv, C, tile=tile | ops.GEMM_BF16, split_k=split)
        assert _rel(C, ref) < 5e-6, (split,)
    # the flag is really applied: the bf16 result is NOT the fp32 product
    assert _rel(C, A.double() @ B.double()) > 1e-4


def test_gemm_bf16_context_epilogue_reduce_batch_and_scatter():
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(3)
    M, N, K = 200, 96, 48
    A = torch.randn(M, K, generator=g).to(DEV)
    W = torch.randn(N, K, generator=g).to(DEV)
    bias = torch.randn(N, generator=g).to(DEV)
    C = torch.randn(M, N, generator=g).to(DEV)
    C0 = C.clone()
    with ops.gemm_precision("bf16"):
        ops.gemm(A, W.t(), C, beta=0.5, bias=bias, relu=True)
    ref = torch.relu(_rb(A) @ _rb(W).t() + 0.5 * C0.double() + bias.double())
    assert _rel(C, ref) < 5e-6
    # context restored: fp32 again afterwards
    C2 = torch.empty(M, N, device=DEV)
    ops.gemm(A, W.t(), C2)
    assert _rel(C2, A.double() @ W.double().t()) < 2e-6
    # batch-reduced weight gradient (shared angle projection) in bf16
    Ab = torch.randn(4, 64, 256, generator=g).to(DEV)
    Bb = torch.randn(4, 256, 96, generator=g).to(DEV)
    Cb = torch.empty(64, 96, device=DEV)
    with ops.gemm_precision("bf16"):
        ops.gemm(Ab, Bb, Cb, reduce_batch=True)
    assert _rel(Cb, (_rb(Ab) @ _rb(Bb)).sum(0)) < 5e-6
    # row scatter
    rows = torch.randperm(300, generator=g)[:M].to(torch.int32).to(DEV)
    Cs = torch.zeros(300, N, device=DEV)
    with ops.gemm_precision("bf16"):
        ops.gemm(A, W.t(), Cs, c_rows=rows)
    assert _rel(Cs[rows.long()], _rb(A) @ _rb(W).t()) < 5e-6
    with pytest.raises(ValueError):
        with ops.gemm_precision("fp16"):
            pass


def test_bf16_training_step_tracks_fp32():
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    res = {}
    for prec in ("fp32", "bf16"):
        torch.manual_seed(0)
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
        tr = A.FusedTrainer(model, precision=prec)
        assert model._engine.precision == prec
        b = mp_like_batch(4).to(DEV)
        loss = tr.forward_backward(b, 5, training=False).clone()
        torch.cuda.synchronize()
        res[prec] = (loss, tr.st.grad.clone())
    (l32, g32), (l16, g16) = res["fp32"], res["bf16"]
    assert torch.isfinite(l16).all() and torch.isfinite(g16).all()
    assert abs(float(l16) - float(l32)) <= 2e-2 * abs(float(l32))
    cos = float((g16.double() @ g32.double()) / (g16.double().norm() * g32.double().norm()))
    assert cos > 0.999, cos
    assert not torch.equal(g16, g32)   # bf16 arithmetic really used
