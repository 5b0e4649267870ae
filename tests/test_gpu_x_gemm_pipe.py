"""Pipelined GEMM main loop (gemm.hip gemm_pipe_kernel: two register sets of global loads in flight)
against the one-stage loop (ALIGNN_GEMM_NOPIPE): same MFMA order and epilogue, so bitwise equal, on
the product shapes of the training step (full stages, vectorisable operands: the pipelined path)
and on shapes that fall back (partial stages, odd strides).  Plus fp64 accuracy of the pipelined
result.  fp32 and bf16 arithmetic."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ops():
    from alignn_mi355x import ops
    return ops


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


CASES = [
    # (M, N, K, batch, layout): the step's products (B = 32) and fallbacks
    (23040, 256, 256, 1, "nt"), (23040, 256, 256, 1, "nn"), (256, 256, 23040, 1, "tn"),
    (2580, 768, 256, 1, "nt"), (2580, 64, 256, 4, "nn"), (64, 256, 2580, 4, "tn"), (1920, 256, 1024, 1, "nn"),
    (2580, 256, 64, 4, "nn"), (300, 257, 129, 1, "nt"), (1000, 96, 48, 2, "tt"),
]


@pytest.mark.parametrize("bf", [False, True])
@pytest.mark.parametrize("M,N,K,batch,layout", CASES)
def test_pipelined_gemm_bitwise_vs_one_stage(M, N, K, batch, layout, bf):
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(M + 3 * N + 7 * K + batch)
    A = torch.randn(batch, M, K, generator=g).to(DEV)
    B = torch.randn(batch, K, N, generator=g).to(DEV)
    Av = A if layout[0] == "n" else A.transpose(1, 2).contiguous().transpose(1, 2)
    Bv = B if layout[1] == "n" else B.transpose(1, 2).contiguous().transpose(1, 2)
    bias = torch.randn(batch, N, generator=g).to(DEV)
    C0 = torch.randn(batch, M, N, generator=g).to(DEV)
    flags = ops.GEMM_BF16 if bf else 0
    outs = []
    for nopipe in (False, True):
        C = C0.clone()
        ops.gemm(Av, Bv, C, beta=1.0, bias=bias, relu=True, tile=flags | (ops.GEMM_NOPIPE if nopipe else 0))
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    if not bf:
        ref = torch.relu(A.double() @ B.double() + C0.double() + bias.double()[:, None, :])
        assert _rel(outs[0], ref) < 5e-6

