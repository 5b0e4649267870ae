"""Skinny products (skinny.hip; the angle encoder's first Linear over T rows, train.py:358-364):
alignn_linear_smallk_f32 and alignn_gemm_tn_smalln_f32 against fp64 torch, including ragged row
counts, non-vector column counts, K = 0 and accumulation; then the engine with
``skinny_encoder`` on vs off (same arithmetic up to fp32 summation order).  Sorts after the core
suites (opt-in path, added after the last on-GPU verification)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


@pytest.mark.parametrize("M,K,N", [(1, 1, 4), (63, 11, 256), (253440 // 8, 11, 256), (1000, 16, 260), (77, 5, 8)])
@pytest.mark.parametrize("relu", [False, True])
def test_linear_smallk(M, K, N, relu):
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(M + 7 * K + N)
    ldx = (K + 3) // 4 * 4
    Xb = torch.randn(M, ldx, generator=g).to(DEV)
    X = Xb[:, :K]
    W = torch.randn(N, K, generator=g).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    out = torch.full((M, N), float("nan"), device=DEV)
    assert ops.linear_smallk_ok(X, W, out)
    ops.linear_smallk(X, W, b, out, relu=relu)
    ref = X.double() @ W.double().t() + b.double()
    if relu:
        ref = ref.clamp(min=0)
    assert torch.isfinite(out).all()
    assert _rel(out, ref) < 1e-6


def test_linear_smallk_rejects_unsupported():
    from alignn_mi355x import ops
    X = torch.randn(10, 17, device=DEV)
    W = torch.randn(8, 17, device=DEV)
    out = torch.empty(10, 8, device=DEV)
    assert not ops.linear_smallk_ok(X, W, out)
    with pytest.raises(ValueError):
        ops.linear_smallk(X, W, None, out)


@pytest.mark.parametrize("K,M,N", [(0, 256, 11), (1, 256, 11), (1000, 256, 11), (253440, 256, 11),
                                   (5000, 130, 16), (777, 37, 3), (64, 256, 0)])
def test_gemm_tn_smalln(K, M, N):
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(K + 3 * M + N)
    A = torch.randn(K, M, generator=g).to(DEV)
    Xb = torch.randn(K, 12 if N <= 12 else N, generator=g).to(DEV)
    X = Xb[:, :N]
    C = torch.full((M, N), float("nan"), device=DEV)
    cs = torch.full((M,), float("nan"), device=DEV)
    ops.gemm_tn_smalln(A, X, C, colsum=cs)
    refC = A.double().t() @ X.double()
    refs = A.double().sum(0)
    if N:
        assert _rel(C, refC) < 2e-6 if K else torch.equal(C, torch.zeros_like(C))
    assert _rel(cs, refs) < 2e-6 if K else torch.equal(cs, torch.zeros_like(cs))
    # accumulate, and determinism
    C2, cs2 = C.clone(), cs.clone()
    ops.gemm_tn_smalln(A, X, C2, colsum=cs2, accumulate=True)
    if K and N:
        assert _rel(C2, 2 * refC) < 2e-6
    C3, cs3 = torch.empty_like(C), torch.empty_like(cs)
    ops.gemm_tn_smalln(A, X, C3, colsum=cs3)
    assert torch.equal(C3, C) and torch.equal(cs3, cs)


def test_engine_skinny_encoder_matches_tiled():
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    res = []
    for skinny in (False, True):
        torch.manual_seed(0)
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
        model._engine.skinny_encoder = skinny
        tr = A.FusedTrainer(model)
        b = mp_like_batch(4).to(DEV)
        loss = tr.forward_backward(b, 3).clone()
        torch.cuda.synchronize()
        res.append((loss, tr.st.grad.clone()))
    (l0, g0), (l1, g1) = res
    assert abs(float(l1) - float(l0)) <= 1e-5 * abs(float(l0))
    assert float((g1 - g0).norm() / g0.norm()) < 1e-5
