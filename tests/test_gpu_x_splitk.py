"""In-launch split-K combine (gemm.hip splitk_combine: each tile's last-arriving workgroup sums the
split partials after an agent-scope release/acquire hand-off on a per-tile ticket) against the
separate reduce launch (ops.SPLITK_COMBINE = False): the same fixed summation order, so bitwise equal
results, on the step's split-K products (weight gradients with K = rows, batch-reduced shared
weights, long-K projections), ragged tiles, beta/bias/scatter epilogues, and repeated launches (the
tickets return to zero after every call)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [
    # (M, N, K, batch, layout, reduce_batch)
    (256, 256, 23040, 1, "tn", False), (64, 256, 2580, 4, "tn", False), (256, 36, 23040, 1, "tn", False),
    (1920, 256, 1024, 1, "nn", False), (256, 256, 256, 4, "nn", True), (100, 70, 5000, 3, "nt", False),
    (256, 206, 1920, 1, "tn", False),
]


@pytest.mark.parametrize("M,N,K,batch,layout,rb", CASES)
@pytest.mark.parametrize("epi", ["plain", "beta_bias", "scatter"])
def test_splitk_combine_bitwise_vs_reduce_launch(M, N, K, batch, layout, rb, epi):
    from alignn_mi355x import _lib, ops
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K + batch)
    A = torch.randn(batch, M, K, generator=g).to(DEV)
    B = torch.randn(batch, K, N, generator=g).to(DEV)
    Av = A if layout[0] == "n" else A.transpose(1, 2).contiguous().transpose(1, 2)
    Bv = B if layout[1] == "n" else B.transpose(1, 2).contiguous().transpose(1, 2)
    if batch == 1:
        Av, Bv = Av[0], Bv[0]
    outb = 1 if (rb or batch == 1) else batch
    shape = (M, N) if outb == 1 else (outb, M, N)
    C0 = torch.randn(*shape, generator=g).to(DEV)
    kw = dict(reduce_batch=rb)
    if epi == "beta_bias":
        kw.update(beta=0.5, bias=torch.randn(N, generator=g).to(DEV) if outb == 1 else
                  torch.randn(outb, N, generator=g).to(DEV))
    if epi == "scatter" and outb == 1:
        kw.update(c_rows=torch.randperm(M, generator=g).to(torch.int32).to(DEV))
    outs = []
    for combine in (True, False, True, True):
        ops.SPLITK_COMBINE, prev = combine, ops.SPLITK_COMBINE_MAX
        ops.SPLITK_COMBINE_MAX = 1 << 20   # every split count (the default limits it to few splits)
        try:
            C = C0.clone()
            ops.gemm(Av, Bv, C, **kw)
        finally:
            ops.SPLITK_COMBINE, ops.SPLITK_COMBINE_MAX = True, prev
        outs.append(C)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    ref = (A.double() @ B.double())
    ref = ref.sum(0) if rb else (ref[0] if outb == 1 else ref)
    if epi == "beta_bias":
        bias = kw["bias"].double()
        ref = ref + 0.5 * C0.double() + (bias[:, None, :] if bias.dim() == 2 else bias)
    if "c_rows" in kw:
        full = C0.double().clone()
        full[kw["c_rows"].long()] = ref
        ref = full
    assert float((outs[0].double() - ref).abs().max() / ref.abs().max()) < 5e-6
    # the plan split K (otherwise this test checks nothing)
    a = _lib.GemmArgs()
    a.M, a.N, a.K, a.batch, a.reduce_batch = M, N, K, batch, int(rb)
    a.sam, a.sak, a.sbk, a.sbn, a.scm, a.scn = K, 1, 1, K, N, 1
    assert _lib.lib().alignn_gemm_counters(__import__("ctypes").byref(a)) > 0
