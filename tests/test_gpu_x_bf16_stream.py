"""bf16 streaming GEMM (gemm.hip gemm_bf16_stream_kernel: a 256-column slice of W in LDS as bf16,
64-row bands of A streamed through registers, v_mfma_f32_32x32x16_bf16) — the kernel config C3's
large-M products take.  Its inputs are rounded to bf16 (RNE) and products accumulate in fp32, so
against an fp64 product of the bf16-rounded operands the error is fp32 accumulation only; against
the tiled bf16 path (ALIGNN_GEMM_NOSTREAM) the two differ by accumulation order.  Shapes of the
B = 256 step plus ragged M, both W layouts, and the epilogue terms it supports.  Below 32768 rows
the kernel is taken only on request (ALIGNN_GEMM_STREAM: inside the C3 plan the tiled kernels win
there), so the smaller cases ask for it; every case turns the row-streaming kernel off
(ALIGNN_GEMM_NOROWS: it takes these shapes first, tests in test_gpu_x_gemm_rows.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


CASES = [(184320, 256, 256, "nt"), (184320, 256, 256, "nn"), (15360, 1024, 256, "nt"), (16020, 768, 256, "nt"),
         (16020, 256, 128, "nn"), (5001, 512, 64, "nt"), (4097, 256, 256, "nn")]


@pytest.mark.parametrize("M,N,K,layout", CASES)
@pytest.mark.parametrize("epi", ["plain", "bias_relu", "beta_bias", "mask"])
def test_bf16_stream_vs_fp64_of_rounded_inputs(M, N, K, layout, epi):
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
    BF = ops.GEMM_BF16 | ops.GEMM_NOROWS | (ops.GEMM_STREAM if M < 32768 else 0)
    kw = dict(beta=beta, bias=bias, relu=relu, mask=mask)
    assert ops.gemm(A, Wv, C0, tile=BF, path_only=True, **kw) == 1
    assert ops.gemm(A, Wv, C0, tile=BF | ops.GEMM_NOSTREAM, path_only=True, **kw) == 0
    C = C0.clone()
    ops.gemm(A, Wv, C, tile=BF, **kw)
    Ct = C0.clone()
    ops.gemm(A, Wv, Ct, tile=BF | ops.GEMM_NOSTREAM, **kw)
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
    assert _rel(C, Ct) < 5e-6
    assert torch.equal(C, C2)   # fixed order, no atomics


def test_bf16_stream_routing_and_untouched_rows():
    from alignn_mi355x import ops
    BF = ops.GEMM_BF16 | ops.GEMM_STREAM | ops.GEMM_NOROWS
    A = torch.randn(8000, 256, device=DEV)
    W = torch.randn(256, 256, device=DEV)
    C = torch.empty(8000, 256, device=DEV)
    assert ops.gemm(A, W, C, tile=BF, path_only=True) == 1
    assert ops.gemm(A, W, C, path_only=True) == 0                                 # fp32: tiled
    assert ops.gemm(A, W, C, tile=ops.GEMM_BF16 | ops.GEMM_NOROWS, path_only=True) == 0   # M < 32768 unasked
    assert ops.gemm(A[:4000], W, C[:4000], tile=BF, path_only=True) == 0          # M < 4096
    assert ops.gemm(A[:, :200], W[:200], C, tile=BF, path_only=True) == 0         # K not 64/128/256
    assert ops.gemm(A, W[:, :200], C[:, :200], tile=BF, path_only=True) == 0      # N % 256
    rows = torch.arange(8000, dtype=torch.int32, device=DEV)
    assert ops.gemm(A, W, C, tile=BF, c_rows=rows, path_only=True) == 0
    assert ops.gemm(A, W, C, tile=BF, mask=C.t().contiguous().t(), path_only=True) == 0   # column-major mask
    # rows past M of the last band are dropped by the store descriptor
    buf = torch.full((4200, 256), 7.0, device=DEV)
    ops.gemm(A[:4100], W, buf[:4100], tile=BF)
    torch.cuda.synchronize()
    assert bool((buf[4100:] == 7.0).all())
