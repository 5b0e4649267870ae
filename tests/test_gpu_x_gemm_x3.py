"""fp32 GEMM as three bf16 words (ALIGNN_GEMM_F32X3): each fp32 operand is split exactly into
hi + mid + lo bf16 words and the six cross products down to 2^-16 of hi*hi run on
v_mfma_f32_32x32x16_bf16 with fp32 accumulation.  Every dropped term is below 2^-24 |a b|, so the
result is fp32-class: checked against an fp64 product next to the exact f32 MFMA path's own error
(north_star: 1e-4 relative to the fp32 CPU path; these products stay near 1e-7)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


@pytest.mark.parametrize("tile", [0, 1, 2, 4, 17, 36, 132])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
def test_gemm_x3_layouts_tiles_splits(tile, layout):
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(tile * 7 + ord(layout[0]) + 3 * ord(layout[1]))
    M, N, K = 300, 257, 1000
    A = torch.randn(M, K, generator=g).to(DEV)
    B = torch.randn(K, N, generator=g).to(DEV)
    Av = A if layout[0] == "n" else A.t().contiguous().t()
    Bv = B if layout[1] == "n" else B.t().contiguous().t()
    ref = A.double() @ B.double()
    for split in (1, 3):
        C = torch.empty(M, N, device=DEV)
        C32 = torch.empty(M, N, device=DEV)
        ops.gemm(Av, Bv, C, tile=tile | ops.GEMM_F32X3, split_k=split)
        ops.gemm(Av, Bv, C32, tile=tile, split_k=split)
        e3, e32 = _rel(C, ref), _rel(C32, ref)
        assert e3 < 2e-6 and e3 < 4 * e32 + 2e-7, (split, e3, e32)
    assert not torch.equal(C, C32)    # the flag is really applied (not the f32 MFMA's bits)


@pytest.mark.parametrize("M,N,K,batch", [(23040, 256, 256, 1), (256, 256, 23040, 1), (64, 256, 2580, 4),
                                         (2580, 64, 256, 4), (33, 17, 5, 1), (1, 256, 1, 4)])
def test_gemm_x3_step_shapes(M, N, K, batch):
    """The training step's product shapes (auto plans: split-K, 64-deep stages, pipelined loop) and
    ragged ones."""
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn(batch, M, K, generator=g).to(DEV)
    B = torch.randn(batch, K, N, generator=g).to(DEV)
    C = torch.empty(batch, M, N, device=DEV)
    C32 = torch.empty(batch, M, N, device=DEV)
    ops.gemm(A, B, C, tile=ops.GEMM_F32X3)
    ops.gemm(A, B, C32)
    ref = A.double() @ B.double()
    e3, e32 = _rel(C, ref), _rel(C32, ref)
    assert e3 < 2e-6 and e3 < 4 * e32 + 2e-7, (e3, e32)


def test_gemm_x3_wide_dynamic_range_epilogue_and_reduce_batch():
    """Rows scaled over 1e-20..1e20 (each word's exponent follows its own value), epilogue terms
    (beta, bias, relu), the batch-reduced weight gradient."""
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(11)
    M, N, K = 200, 96, 300
    scale = torch.logspace(-20, 20, M, dtype=torch.float64).float()
    A = (torch.randn(M, K, generator=g) * scale[:, None]).to(DEV)
    W = torch.randn(N, K, generator=g).to(DEV)
    ref = A.double() @ W.double().t()
    C = torch.empty(M, N, device=DEV)
    ops.gemm(A, W.t(), C, tile=ops.GEMM_F32X3)
    row_err = ((C.double() - ref).abs().amax(1) / ref.abs().amax(1)).max().item()
    assert row_err < 2e-6
    bias = torch.randn(N, generator=g).to(DEV)
    A2 = torch.randn(M, K, generator=g).to(DEV)
    C = torch.randn(M, N, generator=g).to(DEV)
    C0 = C.clone()
    ops.gemm(A2, W.t(), C, beta=0.5, bias=bias, relu=True, tile=ops.GEMM_F32X3)
    assert _rel(C, torch.relu(A2.double() @ W.double().t() + 0.5 * C0.double() + bias.double())) < 2e-6
    Ab = torch.randn(4, 64, 256, generator=g).to(DEV)
    Bb = torch.randn(4, 256, 96, generator=g).to(DEV)
    Cb = torch.empty(64, 96, device=DEV)
    ops.gemm(Ab, Bb, Cb, reduce_batch=True, tile=ops.GEMM_F32X3)
    assert _rel(Cb, (Ab.double() @ Bb.double()).sum(0)) < 2e-6


def test_gemm_x3_nonfinite_inputs_propagate_like_f32():
    """An inf operand gives inf/NaN exactly where the f32 MFMA path does (the split keeps
    mid = lo = 0 for a non-finite hi word), a NaN gives NaN: the GradScaler's found-inf check sees
    the same non-finite gradients."""
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(5)
    M, N, K = 96, 80, 64
    A = torch.randn(M, K, generator=g)
    B = torch.randn(K, N, generator=g).abs() + 0.1   # positive: inf * B stays inf
    A[3, 5] = float("inf")
    A[7, 1] = float("-inf")
    A[9, 2] = float("nan")
    A, B = A.to(DEV), B.to(DEV)
    C = torch.empty(M, N, device=DEV)
    C32 = torch.empty(M, N, device=DEV)
    ops.gemm(A, B, C, tile=ops.GEMM_F32X3)
    ops.gemm(A, B, C32)
    assert torch.equal(torch.isposinf(C), torch.isposinf(C32))
    assert torch.equal(torch.isneginf(C), torch.isneginf(C32))
    assert torch.equal(torch.isnan(C), torch.isnan(C32))
    fin = torch.isfinite(C32)
    assert _rel(C[fin], C32[fin]) < 2e-6
