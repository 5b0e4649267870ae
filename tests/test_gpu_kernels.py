"""GPU unit parity of the individual HIP kernels (through the C ABI) against plain PyTorch fp32 /
integer references.  Run with -m gpu on an MI355X."""
import numpy as np
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


@pytest.mark.parametrize("M,N,K", [(1, 1, 1), (37, 53, 11), (128, 128, 16), (300, 257, 129), (2049, 1024, 256),
                                   (64, 256, 23040)])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
def test_gemm_layouts(M, N, K, layout):
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N * 13 + K)
    A = torch.randn(M, K, generator=g).to(DEV)
    B = torch.randn(K, N, generator=g).to(DEV)
    Av = A if layout[0] == "n" else A.t().contiguous().t()
    Bv = B if layout[1] == "n" else B.t().contiguous().t()
    C = torch.empty(M, N, device=DEV)
    ops.gemm(Av, Bv, C)
    ref = A.double() @ B.double()
    assert _rel(C, ref) < 2e-6


def test_gemm_epilogues_and_batch():
    ops = _ops()
    torch.manual_seed(0)
    H, M, K, N = 4, 300, 64, 256
    A = torch.randn(H, M, K, device=DEV)
    B = torch.randn(H, K, N, device=DEV)
    C0 = torch.randn(H, M, N, device=DEV)
    bias = torch.randn(H, N, device=DEV)
    rs = torch.randn(H, M, device=DEV)
    b2 = torch.randn(H, N, device=DEV)
    C = C0.clone()
    ops.gemm(A, B, C, alpha=0.5, beta=1.0, bias=bias, rowscale=rs, bias2=b2)
    ref = 0.5 * (A.double() @ B.double()) + C0.double() + bias.double()[:, None, :] + rs.double()[:, :, None] * b2.double()[:, None, :]
    assert _rel(C, ref) < 2e-6
    # relu + mask
    X = torch.randn(M, K, device=DEV)
    W = torch.randn(N, K, device=DEV)
    mask = torch.randn(M, N, device=DEV)
    out = torch.empty(M, N, device=DEV)
    ops.gemm(X, W.t(), out, relu=True, mask=mask)
    ref = torch.relu(X.double() @ W.double().t()) * (mask > 0)
    assert _rel(out, ref) < 2e-6


def test_gemm_split_k_deterministic():
    ops = _ops()
    torch.manual_seed(1)
    A = torch.randn(23040, 1024, device=DEV)
    X = torch.randn(23040, 256, device=DEV)
    out1 = torch.empty(1024, 256, device=DEV)
    out2 = torch.empty(1024, 256, device=DEV)
    ops.gemm(A.t(), X, out1, split_k=16)
    ops.gemm(A.t(), X, out2, split_k=16)
    assert torch.equal(out1, out2)
    ref = A.double().t() @ X.double()
    assert _rel(out1, ref) < 5e-6


@pytest.mark.parametrize("M,N,K,batch", [(2580, 768, 256, 1), (23040, 256, 256, 1), (64, 256, 2580, 4),
                                         (2580, 64, 256, 4), (256, 11, 253440, 1), (64, 1, 23040, 4)])
def test_gemm_auto_plan_shapes(M, N, K, batch):
    """The step's GEMM shapes under the library's automatic tile/split-K plan (all four tile shapes,
    split and unsplit) vs fp64."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(M + N + K + batch)
    A = torch.randn(batch, K, M, generator=g).to(DEV).transpose(1, 2)   # m-contiguous A (weight-grad layout)
    B = torch.randn(batch, K, N, generator=g).to(DEV)
    C = torch.empty(batch, M, N, device=DEV)
    ops.gemm(A, B, C)
    ref = A.double() @ B.double()
    assert _rel(C, ref) < 5e-6


def test_gemm_c_rows_scatter():
    ops = _ops()
    torch.manual_seed(3)
    n, na, K, N = 5000, 700, 768, 256
    rows = torch.randperm(n)[:na].sort().values.to(torch.int32).to(DEV)
    A = torch.randn(na, K, device=DEV)
    W = torch.randn(K, N, device=DEV)
    C0 = torch.randn(n, N, device=DEV)
    C = C0.clone()
    ops.gemm(A, W, C, beta=1.0, c_rows=rows)
    ref = C0.double().clone()
    ref[rows.long()] += A.double() @ W.double()
    assert _rel(C, ref) < 2e-6
    # scatter / gather row helpers
    out = torch.zeros(n, N, device=DEV)
    ops.scatter_rows(A[:, :N].contiguous(), rows, out)
    assert torch.equal(out[rows.long()], A[:, :N]) and float(out.abs().sum()) == float(A[:, :N].abs().sum())
    assert torch.equal(ops.gather_rows(out, rows), A[:, :N])


def test_colsum():
    ops = _ops()
    X = torch.randn(100003, 300, device=DEV)
    out = torch.empty(300, device=DEV)
    ops.colsum(X, out)
    assert _rel(out, X.double().sum(0)) < 1e-5


def _edges(n, m, layout, g):
    """[src; dst] lists whose keys repeat within a wave in different ways (the CSR build groups each
    wave's lanes by key): random; a few targets interleaved (as a line graph's sources repeat in
    target order); runs of one target whose sources come in runs of 8; one key throughout."""
    if layout == "random":
        return torch.randint(0, n, (2, m), generator=g)
    i = torch.arange(m)
    if layout == "interleaved":
        return torch.stack([torch.randint(0, n, (m,), generator=g), (i % 12 + 12 * (i // 1200)) % n])
    if layout == "runs":
        return torch.stack([((i % 97) // 8 + 13 * (i // 97)) % n, (i // 97) % n])
    return torch.stack([torch.full((m,), n // 3), torch.full((m,), n // 2)])


@pytest.mark.parametrize("n,m,layout", [(7, 19, "random"), (1000, 20000, "random"), (50, 0, "random"),
                                        (5, 1, "random"), (2580, 253440, "interleaved"), (2580, 253440, "runs"),
                                        (300, 2000, "constant")])
def test_graph_prep_bit_exact(n, m, layout):
    ops = _ops()
    g = torch.Generator().manual_seed(n + m)
    ei = _edges(n, m, layout, g)
    csr = ops.GraphCSR(ei.to(DEV), n)
    torch.cuda.synchronize()
    csr.check_indices("test")
    dst = ei[1].numpy()
    perm = np.argsort(dst, kind="stable")
    off = np.concatenate([[0], np.cumsum(np.bincount(dst, minlength=n))])
    assert np.array_equal(csr.off_dst.cpu().numpy(), off)
    if m:
        assert np.array_equal(csr.perm_dst[:m].cpu().numpy(), perm)
        assert np.array_equal(csr.src_at[:m].cpu().numpy(), ei[0].numpy()[perm])
        assert np.array_equal(csr.dst_at[:m].cpu().numpy(), dst[perm])
        src_sorted = ei[0].numpy()[perm]
        perm2 = np.argsort(src_sorted, kind="stable")
        assert np.array_equal(csr.pos_src[:m].cpu().numpy(), perm2)


def test_graph_prep_flags_out_of_range():
    ops = _ops()
    ei = torch.tensor([[0, 1, 5], [1, 2, 0]], device=DEV)
    csr = ops.GraphCSR(ei, 3)
    with pytest.raises(IndexError):
        csr.check_indices("edge_index")
    # an out-of-range key among lanes that share one in-range key
    ei = torch.stack([torch.zeros(200, dtype=torch.int64), torch.full((200,), 2)]).to(DEV)
    ei[1, 77] = 3
    csr = ops.GraphCSR(ei, 3)
    with pytest.raises(IndexError):
        csr.check_indices("edge_index")


def test_hetero_nll_matches_torch():
    ops = _ops()
    torch.manual_seed(3)
    B, T = 32, 2
    heads = torch.randn(B, 2 * T, device=DEV)
    heads[0, T] = -5.0  # below the logvar floor: clamped, zero gradient
    y = torch.rand(B * T, device=DEV) * 299 + 1
    lm = torch.tensor([4.3228, 3.5567], device=DEV)
    ls = torch.tensor([0.9051, 0.9405], device=DEV)
    loss = torch.zeros(1, device=DEV)
    dh = torch.empty_like(heads)
    ops.hetero_nll(heads, y, lm, ls, -2.9, 0.1, loss, dh)
    h = heads.double().clone().requires_grad_(True)
    mean, logvar = h[:, :T], h[:, T:]
    tz = (torch.log(y.double().view(B, T)) - lm.double()) / ls.double()
    lv = torch.clamp(logvar, min=-2.9)
    ref = (0.5 * (lv + (mean - tz) ** 2 / torch.exp(lv))).mean(1).mean() + 0.1 * (0.5 * lv).pow(2).mean()
    ref.backward()
    assert abs(float(loss) - float(ref)) < 1e-5 * abs(float(ref))
    assert _rel(dh, h.grad) < 1e-5
    assert float(dh[0, T]) == 0.0


def test_dropout_statistics_and_replay():
    ops = _ops()
    x = torch.ones(1000, 1000, device=DEV)
    y1 = torch.empty_like(x)
    y2 = torch.empty_like(x)
    ops.dropout(x, y1, None, 0.15, 1234)
    ops.dropout(x, y2, None, 0.15, 1234)
    assert torch.equal(y1, y2)
    keep = (y1 > 0).float().mean().item()
    assert abs(keep - 0.85) < 0.003
    assert torch.allclose(y1[y1 > 0], torch.full_like(y1[y1 > 0], 1 / 0.85))
    y3 = torch.empty_like(x)
    ops.dropout(x, y3, None, 0.15, 1235)
    assert not torch.equal(y1, y3)


def test_add_noise_moments():
    ops = _ops()
    x = torch.zeros(4_000_000, device=DEV)
    ops.add_noise(x, 0.1, 99)
    assert abs(x.mean().item()) < 5e-4
    assert abs(x.std().item() - 0.1) < 5e-4


@pytest.mark.parametrize("M,N,H", [(1, 64, 1), (37, 256, 4), (2580, 256, 4), (1920, 128, 2), (0, 256, 4)])
def test_wcolsum2_matches_fp64(M, N, H):
    """alignn_wcolsum2_f32 (the per-head w-bar gradient) vs fp64 torch, on strided row views."""
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(M + N + H)
    X1 = torch.randn(M, 3 * N, generator=g).to(DEV)[:, :N]         # a QKV-like row stride
    X2 = torch.randn(M, N, generator=g).to(DEV)
    W1 = torch.randn(M, H, generator=g).to(DEV)
    W2 = torch.randn(M, H, generator=g).to(DEV)
    out = torch.full((N,), float("nan"), device=DEV)
    ops.wcolsum2(X1, W1, X2, W2, out)
    C = N // H
    ref = (X1.double() * W1.double().repeat_interleave(C, 1) + X2.double() * W2.double().repeat_interleave(C, 1)).sum(0)
    torch.cuda.synchronize()
    scale = max(1.0, float(ref.abs().max()))
    assert float((out.double() - ref).abs().max()) <= 1e-5 * scale * max(1, M) ** 0.5
    base = out.clone()
    ops.wcolsum2(X1, W1, X2, W2, out, accumulate=True)
    torch.cuda.synchronize()
    assert torch.allclose(out, 2 * base, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("n,D,H", [(300, 256, 4), (57, 64, 1), (129, 128, 2)])
def test_bwd_src_by_source_list_bitwise(n, D, H):
    """alignn_tconv_bwd_src_by (targets in by-source order, next group's indices prefetched, clamped
    tails) against alignn_tconv_bwd_src: the same sums in the same order, bit for bit; and against
    an fp64 scatter of the per-edge terms.  Ragged out-degrees: 0, 1, 16, 17, up to 140."""
    from alignn_mi355x import _lib, ops
    g = torch.Generator(device="cpu").manual_seed(n + D)
    outdeg = torch.randint(0, 141, (n,), generator=g)
    outdeg[::7] = 0
    outdeg[1], outdeg[2], outdeg[3] = 1, 16, 17
    src = torch.repeat_interleave(torch.arange(n), outdeg)
    dst = torch.randint(0, n, (src.numel(),), generator=g)
    perm = torch.randperm(src.numel(), generator=g)
    ei = torch.stack([src[perm], dst[perm]]).to(DEV)
    csr = ops.GraphCSR(ei, n)
    m = csr.m
    QKVR = torch.randn(n, 4 * D, generator=g).to(DEV)
    dout = torch.randn(n, D, generator=g).to(DEV)
    dz = torch.randn(m, H, generator=g).to(DEV)
    al = torch.randn(m, H, generator=g).to(DEV)
    outs = []
    for by in (False, True):
        dKV = torch.full((n, 2 * D), float("nan"), device=DEV)
        ops.tconv_bwd_src(csr, D, H, QKVR, dout, dz, al, dKV, by_source=by)
        outs.append(dKV)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    # fp64: edge position t (target-sorted) has source src_at[t], target dst_at[t]
    s_t = csr.src_at[:m].long().cpu()
    d_t = csr.dst_at[:m].long().cpu()
    C = D // H
    dzr = dz.double().cpu().repeat_interleave(C, 1)
    alr = al.double().cpu().repeat_interleave(C, 1)
    dK = torch.zeros(n, D, dtype=torch.float64).index_add_(0, s_t, dzr * QKVR.double().cpu()[d_t, :D])
    dV = torch.zeros(n, D, dtype=torch.float64).index_add_(0, s_t, alr * dout.double().cpu()[d_t])
    ref = torch.cat([dK, dV], 1)
    assert float((outs[1].double().cpu() - ref).abs().max() / ref.abs().max()) < 1e-5
