"""Register-direct fp32 GEMM (gemm_reg.hip: one wave per output tile, k-contiguous fragments loaded
straight into VGPRs) against the tiled kernels (ALIGNN_GEMM_NOREG): same k-slot assignment, MFMA
order and epilogue, so bitwise equal — on the step's X·Wᵀ shapes, ragged M / N, a batch, a scatter
(c_rows) and a ReLU-backward mask; plus fp64 accuracy.  Shapes the kernel does not take (K % 64,
split-K plans) fall back to the tiled kernels and must still agree."""
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
    # (M, N, K, batch): the step's X·Wᵀ products (B = 32), ragged tiles, a batch, fallbacks
    (23040, 256, 256, 1), (23040, 768, 256, 1), (2580, 768, 256, 1), (9001, 257, 128, 1),
    (1000, 96, 64, 3), (333, 40, 192, 1), (23040, 256, 80, 1), (64, 32, 64, 1),
]


@pytest.mark.parametrize("mode", [1, 2, 3])
@pytest.mark.parametrize("M,N,K,batch", CASES)
def test_reg_gemm_bitwise_vs_tiled(M, N, K, batch, mode):
    ops = _ops()
    flag = {1: ops.GEMM_REG, 2: ops.GEMM_REG2, 3: ops.GEMM_REG | ops.GEMM_REG2}[mode]
    g = torch.Generator(device="cpu").manual_seed(M + 3 * N + 7 * K + batch + mode)
    A = torch.randn(batch, M, K, generator=g).to(DEV)
    W = torch.randn(batch, N, K, generator=g).to(DEV)          # nn.Linear weight [out, in]
    bias = torch.randn(batch, N, generator=g).to(DEV)
    C0 = torch.randn(batch, M, N, generator=g).to(DEV)
    outs = []
    for f in (ops.GEMM_NOREG, flag):
        C = C0.clone()
        ops.gemm(A, W.transpose(1, 2), C, beta=1.0, bias=bias, relu=True, tile=f)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = torch.relu(A.double() @ W.double().transpose(1, 2) + C0.double() + bias.double()[:, None, :])
    assert _rel(outs[1], ref) < 5e-6


@pytest.mark.parametrize("mode", [1, 2])
def test_reg_gemm_scatter_and_mask_bitwise(mode):
    ops = _ops()
    flag = ops.GEMM_REG if mode == 1 else ops.GEMM_REG2
    M, N, K = 5000, 256, 256
    g = torch.Generator(device="cpu").manual_seed(11 + mode)
    A = torch.randn(M, K, generator=g).to(DEV)
    W = torch.randn(N, K, generator=g).to(DEV)
    mask = torch.randn(M, N, generator=g).to(DEV)
    rows = torch.randperm(M + 17, generator=g)[:M].to(torch.int32).to(DEV)
    C0 = torch.randn(M + 17, N, generator=g).to(DEV)
    outs = []
    for f in (ops.GEMM_NOREG, flag):
        C = C0.clone()
        ops.gemm(A, W.t(), C, alpha=0.5, beta=1.0, mask=mask, c_rows=rows, tile=f)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = C0.double().clone()
    v = 0.5 * (A.double() @ W.double().t()) + C0.double()[rows.long()]
    ref[rows.long()] = torch.where(mask > 0, v, torch.zeros_like(v))
    assert _rel(outs[1], ref) < 5e-6
