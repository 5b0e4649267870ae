"""bf16 row-streaming GEMM (csrc/gemm_rows.hip: each wave's 32 columns of W as MFMA operands in VGPRs,
32-row bands of A streamed through double-buffered LDS images, v_mfma_f32_32x32x16_bf16) — the kernel
config C3's bond-level products take (every bond times a 256-wide weight: the skip projection, the
dX += dR W product, the edge MLP).  Same operand rounding (bf16 RNE), k grouping (16-deep slices,
k = 16 t + 8 h + j) and epilogue order as the tiled bf16 kernels, so it is compared with them
bitwise (ALIGNN_GEMM_NOROWS), and with an fp64 product of the rounded
operands to fp32 accumulation error.  Shapes of the B = 256 step (K = 36 the edge MLP's first
layer: zero-padded to 64), ragged M, both W layouts, bf16 A / C storage and every epilogue term it
supports; below 4096 rows the kernel runs on request (ALIGNN_GEMM_ROWS)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


CASES = [(184320, 256, 256, "nt"), (184320, 256, 256, "nn"), (184320, 256, 36, "nt"), (15360, 1024, 256, "nt"),
         (16020, 768, 256, "nn"), (5001, 512, 64, "nt"), (4097, 256, 200, "nn"), (33, 256, 8, "nt")]


@pytest.mark.parametrize("M,N,K,layout", CASES)
@pytest.mark.parametrize("epi", ["plain", "bias_relu", "beta_bias", "mask"])
def test_rows_kernel_matches_tiled_bitwise(M, N, K, layout, epi):
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(DEV)
    W = torch.randn(K, N, generator=g).to(DEV)
    Wv = W if layout[1] == "n" else W.t().contiguous().t()
    bias = torch.randn(N, generator=g).to(DEV) if epi != "plain" else None
    beta = 0.75 if epi == "beta_bias" else 0.0
    relu = epi == "bias_relu"
    C0 = torch.randn(M, N, generator=g).to(DEV)
    mask = torch.randn(M, N, generator=g).to(DEV) if epi == "mask" else None
    BF = ops.GEMM_BF16 | (ops.GEMM_ROWS if M < 4096 else 0)
    kw = dict(beta=beta, bias=bias, relu=relu, mask=mask)
    assert ops.gemm(A, Wv, C0, tile=BF, path_only=True, **kw) == 2
    C = C0.clone()
    ops.gemm(A, Wv, C, tile=BF, **kw)
    Ct = C0.clone()
    ops.gemm(A, Wv, Ct, tile=ops.GEMM_BF16 | ops.GEMM_NOROWS, **kw)
    C2 = C0.clone()
    ops.gemm(A, Wv, C2, tile=BF, **kw)
    torch.cuda.synchronize()
    ref = A.bfloat16().double() @ W.bfloat16().double() + beta * C0.double()
    if bias is not None:
        ref = ref + bias.double()
    if relu:
        ref = torch.relu(ref)
    if mask is not None:
        ref = torch.where(mask > 0, ref, torch.zeros_like(ref))
    assert _rel(C, ref) < 5e-6
    assert torch.equal(C, Ct)
    assert torch.equal(C, C2)   # fixed order, no atomics


@pytest.mark.parametrize("io", ["A16_C16", "A16_beta", "C16", "A16_mask"])
def test_rows_kernel_bf16_storage(io):
    """bf16 A rows (the skip projection reads X16, dX += dR W reads the bf16 dR) and bf16 C (R)."""
    from alignn_mi355x import ops
    M, N, K = 184320, 256, 256
    g = torch.Generator(device="cpu").manual_seed(7)
    A = torch.randn(M, K, generator=g).to(DEV)
    W = (torch.randn(N, K, generator=g) * 0.1).to(DEV)
    bias = torch.randn(N, generator=g).to(DEV)
    A16 = A.bfloat16() if "A16" in io else A
    beta = 1.0 if "beta" in io else 0.0
    mask = torch.randn(M, N, generator=g).to(DEV) if "mask" in io else None
    C0 = torch.randn(M, N, generator=g).to(DEV)
    if "C16" in io:
        C0 = C0.bfloat16()
    kw = dict(beta=beta, bias=None if beta else bias, mask=mask)
    with ops.gemm_precision("bf16"):
        assert ops.gemm(A16, W.t(), C0, path_only=True, **kw) == 2
        C = C0.clone()
        ops.gemm(A16, W.t(), C, **kw)
        Ct = C0.clone()
        ops.gemm(A16, W.t(), Ct, tile=ops.GEMM_NOROWS, **kw)
    torch.cuda.synchronize()
    assert torch.equal(C, Ct)


def test_rows_kernel_routing_and_untouched_rows():
    from alignn_mi355x import ops
    BF = ops.GEMM_BF16 | ops.GEMM_ROWS
    A = torch.randn(8000, 256, device=DEV)
    W = torch.randn(256, 256, device=DEV)
    C = torch.empty(8000, 256, device=DEV)
    assert ops.gemm(A, W, C, tile=BF, path_only=True) == 2
    assert ops.gemm(A, W, C, path_only=True) == 0                                   # fp32 arithmetic: tiled
    assert ops.gemm(A, W, C, tile=ops.GEMM_BF16, path_only=True) == 2               # M >= 4096
    assert ops.gemm(A[:4000], W, C[:4000], tile=ops.GEMM_BF16, path_only=True) == 0  # M < 4096 unasked
    assert ops.gemm(A, W, C, tile=BF | ops.GEMM_NOROWS, path_only=True) == 0
    assert ops.gemm(A[:, :252], W[:252], C, tile=BF, path_only=True) == 2           # K <= 256, K % 4 == 0
    A2, W2 = torch.randn(8000, 260, device=DEV), torch.randn(260, 256, device=DEV)
    assert ops.gemm(A2, W2, C, tile=BF, path_only=True) == 0                        # K > 256
    assert ops.gemm(A, W[:, :200], C[:, :200], tile=BF, path_only=True) == 0        # N % 256
    rows = torch.arange(8000, dtype=torch.int32, device=DEV)
    assert ops.gemm(A, W, C, tile=BF, c_rows=rows, path_only=True) == 0
    assert ops.gemm(A, W, C, tile=BF, mask=C.t().contiguous().t(), path_only=True) == 0   # column-major mask
    # rows past M of the last band are dropped by the store descriptor
    buf = torch.full((4200, 256), 7.0, device=DEV)
    ops.gemm(A[:4100], W, buf[:4100], tile=BF)
    torch.cuda.synchronize()
    assert bool((buf[4100:] == 7.0).all())


@pytest.mark.parametrize("M,lda", [(16020, 768), (15360, 256)])
@pytest.mark.parametrize("a16", [False, True])
def test_rows_kernel_batched_per_head_products(M, lda, a16):
    """The per-head products U_h = Q_h M_h / Vd_h = dout_h M_h (batch = 4 heads, K = 64 columns of a
    wider row, W = M_h row-major [64, 256], C rows of [n, H, D]): each batch entry its own operands."""
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(M + lda)
    X = torch.randn(M, lda, generator=g).to(DEV)
    if a16:
        X = X.bfloat16()
    A = X[:, :256].view(M, 4, 64).transpose(0, 1)            # (4, M, 64), strides (64, lda, 1)
    Mh = (torch.randn(4, 64, 256, generator=g) * 0.1).to(DEV)
    C = torch.full((M, 4, 256), float("nan"), device=DEV)
    Ct = torch.full((M, 4, 256), float("nan"), device=DEV)
    with ops.gemm_precision("bf16"):
        assert ops.gemm(A, Mh, C.transpose(0, 1), path_only=True) == 2
        ops.gemm(A, Mh, C.transpose(0, 1))
        ops.gemm(A, Mh, Ct.transpose(0, 1), tile=ops.GEMM_NOROWS)
    torch.cuda.synchronize()
    ref = torch.einsum("bmk,bkn->mbn", A.bfloat16().double(), Mh.bfloat16().double())
    assert _rel(C, ref) < 5e-6
    assert torch.equal(C, Ct)


@pytest.mark.parametrize("M,ldc", [(16020, 256), (15360, 768)])
@pytest.mark.parametrize("with_proj", [True, False])
def test_heads_kernel_per_head_64_columns(M, ldc, with_proj):
    """The per-head products outp_h += S_h M_h^T (+ sumA_h wbar_h) / dQ_h += Sz_h M_h^T (+ sigz_h
    wbar_h): batch = 4 heads of 64 columns, A_h = S[:, h, :] (K = 256), W_h = M_h^T k-contiguous,
    C rows of [n, H, 64] inside a wider row, beta = 1, the rowscale x bias2 term — bitwise equal
    to the tiled kernels."""
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(M + ldc)
    S = torch.randn(M, 4, 256, generator=g).to(DEV)
    Mh = (torch.randn(4, 64, 256, generator=g) * 0.1).to(DEV)
    out0 = torch.randn(M, ldc, generator=g).to(DEV)
    sumA = torch.rand(M, 4, generator=g).to(DEV)
    wbar = torch.randn(256, generator=g).to(DEV)
    A, B = S.transpose(0, 1), Mh.transpose(1, 2)
    kw = dict(beta=1.0)
    if with_proj:
        kw.update(rowscale=sumA.t(), bias2=wbar.view(4, 64))
    C, Ct = out0.clone(), out0.clone()
    with ops.gemm_precision("bf16"):
        Cv = C[:, :256].view(M, 4, 64).transpose(0, 1)
        assert ops.gemm(A, B, Cv, path_only=True, **kw) == 2
        ops.gemm(A, B, Cv, **kw)
        ops.gemm(A, B, Ct[:, :256].view(M, 4, 64).transpose(0, 1), tile=ops.GEMM_NOROWS, **kw)
    torch.cuda.synchronize()
    ref = torch.einsum("bmk,bkn->mbn", A.bfloat16().double(), B.bfloat16().double()).reshape(M, 256)
    ref = ref + out0[:, :256].double()
    if with_proj:
        ref = ref + (sumA.double()[:, :, None] * wbar.double().view(1, 4, 64)).reshape(M, 256)
    assert _rel(C[:, :256], ref) < 5e-6
    assert torch.equal(C, Ct)   # columns past the heads' 256 untouched on both paths
