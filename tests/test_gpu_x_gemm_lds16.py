"""bf16 LDS images for the bf16 tiled GEMM (gemm_tile.h arithmetic 2: operands rounded to bf16 RNE as
they are staged, one 16-byte LDS read per MFMA fragment, row-contiguous operands transposed into a
[row][k] image by 2-byte stores) against the fp32 LDS images of arithmetic 1, which round the same
values at each fragment read: the MFMA inputs, their order and the epilogue are the same, so bitwise
equal — over every layout, ragged tiles, split-K, batch reduction, the pipelined and the one-stage
loop, bf16 storage of A / B / C, and every tile shape."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ops():
    from alignn_mi355x import ops
    return ops


CASES = [
    # (M, N, K, batch, layout): C3's mid-size products, fallbacks, ragged shapes
    (15360, 256, 256, 1, "nt"), (16020, 256, 768, 1, "nn"), (16020, 768, 256, 1, "nt"),
    (1024, 256, 15360, 1, "tn"), (2580, 64, 256, 4, "nn"), (300, 257, 129, 1, "nt"), (1000, 96, 48, 2, "tt"),
    (777, 130, 200, 1, "tn"),
]


def _mats(M, N, K, batch, layout, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    A = torch.randn(batch, M, K, generator=g).to(DEV)
    B = torch.randn(batch, K, N, generator=g).to(DEV)
    Av = A if layout[0] == "n" else A.transpose(1, 2).contiguous().transpose(1, 2)
    Bv = B if layout[1] == "n" else B.transpose(1, 2).contiguous().transpose(1, 2)
    return g, Av, Bv


@pytest.mark.parametrize("extra", [0, "nopipe", 1, 2, 3, 4, 4 + 128])
@pytest.mark.parametrize("M,N,K,batch,layout", CASES)
def test_lds16_bitwise_vs_fp32_images(M, N, K, batch, layout, extra):
    ops = _ops()
    g, Av, Bv = _mats(M, N, K, batch, layout, M + 3 * N + 7 * K + batch)
    bias = torch.randn(batch, N, generator=g).to(DEV)
    C0 = torch.randn(batch, M, N, generator=g).to(DEV)
    base = ops.GEMM_BF16 | (ops.GEMM_NOPIPE if extra == "nopipe" else (0 if extra in (0, "nopipe") else extra))
    outs = []
    for f in (ops.GEMM_NOLDS16, ops.GEMM_LDS16):
        C = C0.clone()
        ops.gemm(Av, Bv, C, beta=1.0, bias=bias, relu=True, tile=base | f)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = torch.relu(Av.double() @ Bv.double() + C0.double() + bias.double()[:, None, :])
    assert float((outs[1].double() - ref).abs().max() / ref.abs().max()) < 3e-2


@pytest.mark.parametrize("split", [2, 8])
def test_lds16_split_k_and_reduce_batch_bitwise(split):
    ops = _ops()
    g, Av, Bv = _mats(256, 256, 4096, 1, "tn", 5 + split)
    outs = []
    for f in (ops.GEMM_NOLDS16, ops.GEMM_LDS16):
        C = torch.zeros(1, 256, 256, device=DEV)
        ops.gemm(Av, Bv, C, split_k=split, tile=ops.GEMM_BF16 | f)
        outs.append(C)
    _, A3, B3 = _mats(64, 96, 512, 4, "tn", 9 + split)
    for f in (ops.GEMM_NOLDS16, ops.GEMM_LDS16):
        C = torch.zeros(64, 96, device=DEV)
        ops.gemm(A3, B3, C, reduce_batch=True, tile=ops.GEMM_BF16 | f)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[2], outs[3])


@pytest.mark.parametrize("which", ["A", "B", "AC", "ABC"])
def test_lds16_bf16_storage_bitwise(which):
    ops = _ops()
    M, N, K = 4000, 256, 256
    g, Av, Bv = _mats(M, N, K, 1, "nt", 17 + len(which))
    Av, Bv = Av[0], Bv[0]
    if "A" in which:
        Av = Av.bfloat16()
    if "B" in which:
        Bv = Bv.t().contiguous().bfloat16().t()
    outs = []
    for f in (ops.GEMM_NOLDS16, ops.GEMM_LDS16):
        C = torch.zeros(M, N, device=DEV, dtype=torch.bfloat16 if "C" in which else torch.float32)
        ops.gemm(Av, Bv, C, tile=ops.GEMM_BF16 | ops.GEMM_NOROWS | f)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
