"""GPU tests of paths added after the last on-GPU verification (opt-in in the product until they
pass here): the 32-deep GEMM stage and the forward side-stream overlap.  Kept in a file that sorts
after the core parity suites so a failure here cannot stop those under ``pytest -x``."""
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


def _setup(seed=0):
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    torch.manual_seed(seed)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
    tr = A.FusedTrainer(model)
    b = mp_like_batch(4).to(DEV)
    return model, tr, b


@pytest.mark.parametrize("shape", [1, 2, 3, 4])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
def test_gemm_bk32_stage(shape, layout):
    """32-deep K stage (tile bit 4) on every tile shape and operand layout, unsplit and split-K."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(shape * 11 + len(layout))
    M, N, K = 300, 257, 1000
    A = torch.randn(M, K, generator=g).to(DEV)
    B = torch.randn(K, N, generator=g).to(DEV)
    Av = A if layout[0] == "n" else A.t().contiguous().t()
    Bv = B if layout[1] == "n" else B.t().contiguous().t()
    ref = A.double() @ B.double()
    for split in (1, 3):
        C = torch.empty(M, N, device=DEV)
        ops.gemm(Av, Bv, C, tile=16 + shape, split_k=split)
        assert _rel(C, ref) < 5e-6, (split,)
    # batch-reduced (shared weights): K multiple of 32 keeps the 32-deep stage inside one batch entry
    Ab = torch.randn(4, 64, 256, generator=g).to(DEV)
    Bb = torch.randn(4, 256, 96, generator=g).to(DEV)
    Cb = torch.empty(64, 96, device=DEV)
    ops.gemm(Ab, Bb, Cb, reduce_batch=True, tile=16 + shape)
    assert _rel(Cb, (Ab.double() @ Bb.double()).sum(0)) < 5e-6



def test_forward_side_stream_is_bitwise_neutral():
    """The line blocks' skip projection on the side stream (overlap_forward) changes no bits."""
    _, tr1, b1 = _setup()
    _, tr2, b2 = _setup()
    tr2.model._engine.overlap_forward = True
    l1 = tr1.forward_backward(b1, 9)
    l2 = tr2.forward_backward(b2, 9)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2)
    assert torch.equal(tr1.st.grad, tr2.st.grad)
