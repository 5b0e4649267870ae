"""bf16 weight-gradient GEMM (csrc/gemm_wgrad.hip): dW = dY^T X over a long row axis with A = dY^T and
B = X stored row-major over the rows (the layout every Linear's weight gradient has), whole 256 x 256
output tiles per 8-wave workgroup over row chunks, MFMA operands from bf16 LDS images through the
gfx950 transposed read (ds_read_b64_tr_b16), partials through the library's fixed-order split-K
reduce; the bias gradient (rowsum) from the same launch.  Config C3's shapes (184,320 bonds, 15,360
atoms, 16,020 active bonds; bf16 and fp32 storage), ragged ones, the epilogue terms the reduce
applies.  Against an fp64 product of the bf16-rounded operands (fp32 accumulation error only) and the
tiled kernel (ALIGNN_GEMM_NOWGRAD: another summation order)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


CASES = [(256, 256, 184320, "AB"), (256, 256, 184320, "A"), (256, 256, 184320, ""), (256, 36, 184320, ""),
         (1024, 256, 15360, ""), (768, 256, 16020, ""), (264, 40, 4109, "A"), (520, 296, 9000, "B")]


@pytest.mark.parametrize("M,N,K,io", CASES)
def test_wgrad_kernel_vs_fp64_and_tiled(M, N, K, io):
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    dY = torch.randn(K, M, generator=g).to(DEV)
    X = torch.randn(K, N, generator=g).to(DEV)
    if "A" in io:
        dY = dY.bfloat16()
    if "B" in io:
        X = X.bfloat16()
    A = dY.t()
    C = torch.full((M, N), float("nan"), device=DEV)
    Ct = torch.full((M, N), float("nan"), device=DEV)
    rs = torch.full((M,), float("nan"), device=DEV)
    rt = torch.full((M,), float("nan"), device=DEV)
    with ops.gemm_precision("bf16"):
        assert ops.gemm(A, X, C, rowsum=rs, path_only=True) == 3
        assert ops.gemm(A, X, C, rowsum=rs, tile=ops.GEMM_NOWGRAD, path_only=True) == 0
        ops.gemm(A, X, C, rowsum=rs)
        ops.gemm(A, X, Ct, rowsum=rt, tile=ops.GEMM_NOWGRAD)
        C2, rs2 = torch.empty_like(C), torch.empty_like(rs)
        ops.gemm(A, X, C2, rowsum=rs2)
    torch.cuda.synchronize()
    ref = dY.bfloat16().double().t() @ X.bfloat16().double()
    ref_rs = dY.double().sum(0)
    tol = 2e-6 * max(1.0, (K / 1000) ** 0.5)
    assert _rel(C, ref) < tol, _rel(C, ref)
    assert _rel(C, Ct) < tol
    assert _rel(rs, ref_rs) < tol and _rel(rt, ref_rs) < tol
    assert torch.equal(C, C2) and torch.equal(rs, rs2)   # fixed order, no atomics


def test_wgrad_kernel_epilogue_and_routing():
    from alignn_mi355x import ops
    K, M, N = 8192, 256, 256
    g = torch.Generator(device="cpu").manual_seed(5)
    dY, X = torch.randn(K, M, generator=g).to(DEV), torch.randn(K, N, generator=g).to(DEV)
    C0 = torch.randn(M, N, generator=g).to(DEV)
    bias = torch.randn(N, generator=g).to(DEV)
    C = C0.clone()
    with ops.gemm_precision("bf16"):
        ops.gemm(dY.t(), X, C, alpha=0.5, beta=2.0, bias=bias)
        assert ops.gemm(dY.t(), X, C, path_only=True) == 3
        assert ops.gemm(dY.t()[:, :4000], X[:4000], C, path_only=True) == 0        # K < 4096
        assert ops.gemm(dY.t().contiguous(), X, C, path_only=True) == 0           # A k-contiguous
        assert ops.gemm(dY.t(), X, C, mask=C0, path_only=True) == 0
        assert ops.gemm(dY.t(), X, C, split_k=8, path_only=True) == 0
        assert ops.gemm(dY.t()[:64], X, C[:64], path_only=True) == 0                 # M < 128
    assert ops.gemm(dY.t(), X, C, path_only=True) == 0                             # fp32 arithmetic
    torch.cuda.synchronize()
    ref = 0.5 * (dY.bfloat16().double().t() @ X.bfloat16().double()) + 2.0 * C0.double() + bias.double()
    assert _rel(C, ref) < 1e-5


@pytest.mark.parametrize("K,ldq", [(16020, 768), (15360, 1024), (16020, 512)])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_wgrad_kernel_batched_per_head_dM(K, ldq, beta):
    """Batched products (batch = 4 heads, one head's columns of a wider row, N = 256, K = the
    targets), as the per-head edge-projection gradients dM_h = Q_h^T Sz_h (+ dout_h^T S_h, beta = 1)
    with M = 128 (the step's M = 64 ones stay tiled: slower here)."""
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(K + ldq)
    Q = torch.randn(K, ldq, generator=g).to(DEV)
    Sz = torch.randn(K, 4, 256, generator=g).to(DEV)
    A = Q[:, :512].view(K, 4, 128).permute(1, 2, 0)             # (4, 128, K), strides (128, 1, ldq)
    B = Sz.transpose(0, 1)                                      # (4, K, 256), strides (256, 1024, 1)
    C0 = torch.randn(4, 128, 256, generator=g).to(DEV)
    C, Ct = C0.clone(), C0.clone()
    with ops.gemm_precision("bf16"):
        assert ops.gemm(A, B, C, beta=beta, path_only=True) == 3
        ops.gemm(A, B, C, beta=beta)
        ops.gemm(A, B, Ct, beta=beta, tile=ops.GEMM_NOWGRAD)
    torch.cuda.synchronize()
    ref = torch.einsum("bmk,bkn->bmn", A.bfloat16().double(), B.bfloat16().double()) + beta * C0.double()
    tol = 2e-6 * max(1.0, (K / 1000) ** 0.5)
    assert _rel(C, ref) < tol and _rel(C, Ct) < tol
