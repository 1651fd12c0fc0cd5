"""Classifier head fused into the last hidden forward GEMM (gemm_q.hip
EPI_BIAS_RELU_HEAD + head.hip head_xent_parts / head_dgrad_stream) against fp32
PyTorch references of the same ops."""
import pytest
import torch

import ldnn
from ldnn.ops import _ext

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K", [(512, 512, 256), (300, 1000, 200), (4096, 4096, 1024)])
def test_gemm_head_partials_match_fp32(M, N, K):
    C = _ext.C()
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, K, device="cuda", generator=g).bfloat16()
    w = (torch.randn(N, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda", generator=g) * 0.1
    hw = torch.zeros(16, N, device="cuda", dtype=torch.bfloat16)
    hw[:10] = (torch.randn(10, N, device="cuda", generator=g) / N ** 0.5).bfloat16()
    h = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    parts = torch.full(((N + 255) // 256, M, 16), float("nan"), device="cuda")
    C.gemm(x, w, h, True, True, C.EPI_BIAS_RELU, bias=b, head_w=hw, head_part=parts)
    h_ref = torch.relu(x.float() @ w.float().t() + b)
    torch.testing.assert_close(h.float(), h_ref, rtol=2e-2, atol=2e-2)
    # the partial logits are the product of the STORED bf16 activation
    logit_ref = h.float() @ hw.float().t()
    got = parts.sum(0)
    assert torch.isfinite(parts).all()
    torch.testing.assert_close(got, logit_ref, rtol=1e-3, atol=1e-3 * logit_ref.abs().max().item())
    # each 256-column tile's partial is its own slab
    for s in range(parts.shape[0]):
        sl = slice(256 * s, min(N, 256 * (s + 1)))
        ref_s = h[:, sl].float() @ hw[:, sl].float().t()
        torch.testing.assert_close(parts[s], ref_s, rtol=1e-3, atol=1e-3 * max(1.0, ref_s.abs().max().item()))


def test_head_xent_parts_and_dgrad_stream_match_fp32():
    C = _ext.C()
    B, K, ncls = 1000, 512, 10
    g = torch.Generator(device="cuda").manual_seed(1)
    parts = torch.randn(3, B, 16, device="cuda", generator=g)
    parts[:, :, ncls:] = 0
    bias = torch.zeros(16, device="cuda")
    bias[:ncls] = torch.randn(ncls, device="cuda", generator=g) * 0.1
    y = torch.randint(0, ncls, (B,), device="cuda", generator=g)
    logits = torch.empty(B, 16, device="cuda", dtype=torch.bfloat16)
    dlogits = torch.empty(B, 16, device="cuda", dtype=torch.bfloat16)
    stats = torch.zeros((B + 15) // 16, 2, device="cuda")
    C.head_xent_parts(parts, bias, y, logits, dlogits, stats, ncls, 1.0 / B)
    z = (parts.sum(0) + bias)[:, :ncls].bfloat16().float()
    torch.testing.assert_close(logits[:, :ncls].float(), z, rtol=0, atol=0)
    loss = torch.nn.functional.cross_entropy(z, y, reduction="sum")
    assert abs(stats[:, 0].sum().item() - loss.item()) < 1e-3 * max(1.0, loss.item())
    assert int(stats[:, 1].sum().item()) == int((z.argmax(1) == y).sum().item())
    dz = (torch.softmax(z, 1) - torch.nn.functional.one_hot(y, ncls)) / B
    torch.testing.assert_close(dlogits[:, :ncls].float(), dz, rtol=1e-2, atol=1e-5)
    assert (dlogits[:, ncls:] == 0).all()
    # dh = (dlogits W) * relu'(h), dbias += column sums
    h = torch.relu(torch.randn(B, K, device="cuda", generator=g)).bfloat16()
    W = torch.zeros(16, K, device="cuda", dtype=torch.bfloat16)
    W[:ncls] = torch.randn(ncls, K, device="cuda", generator=g).bfloat16()
    dh = torch.empty(B, K, device="cuda", dtype=torch.bfloat16)
    db = torch.zeros(K, device="cuda")
    C.head_dgrad_stream(h, W, dlogits, dh, db, C.EPI_DRELU)
    dh_ref = (dlogits.float() @ W.float()) * (h.float() > 0)
    torch.testing.assert_close(dh.float(), dh_ref, rtol=1e-2, atol=1e-6)
    torch.testing.assert_close(db, dh.float().sum(0), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_engine_fused_head_matches_separate_head(opt):
    """The engine with the head's logits computed in the last hidden forward's epilogue
    trains like the engine running the separate head kernel (partial tiles: hidden 1000,
    batch 4000)."""
    from ldnn.models.mlp import mlp3
    from ldnn.train.static_mlp import OptimConfig, StaticMLPEngine

    torch.manual_seed(0)
    B = 4000
    m1, m2 = mlp3(784, 1000, 10), mlp3(784, 1000, 10)
    m2.load_state_dict(m1.state_dict())
    cfg = OptimConfig(opt, lr=0.05 if opt == "sgd" else 1e-3, momentum=0.9)
    e1 = StaticMLPEngine(m1, B, cfg, use_graphs=True)
    e2 = StaticMLPEngine(m2, B, cfg, use_graphs=True, fuse_head_fwd=False)
    assert e1._head_part is not None and e2._head_part is None
    g = torch.Generator(device="cuda").manual_seed(3)
    l1, l2 = [], []
    for _ in range(5):
        x = torch.randn(B, 784, device="cuda", generator=g).bfloat16()
        y = torch.randint(0, 10, (B,), device="cuda", generator=g)
        for e, ls in ((e1, l1), (e2, l2)):
            e.reset_stats()
            e.load_batch(x, y)
            e.step()
            ls.append(e.read_stats(B))
    for a, b in zip(l1, l2):
        assert abs(a[0] - b[0]) < 1e-3 * max(1.0, abs(b[0])), (l1, l2)
        assert abs(a[1] - b[1]) <= 0.5, (l1, l2)   # accuracy, percent
    # Adam: a gradient element near zero can flip sign between two summation orders (the
    # GPU atomics' arrival order differs run to run), moving its weight by 2 lr per step
    atol = 1e-4 if opt == "sgd" else 5 * cfg.lr
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-3, atol=atol)


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_engine_fused_head_bwd_matches_separate(opt):
    """The engine's fused MFMA head backward (head_bwd: dgrad + wgrad in one pass) trains
    like the head dgrad stream + head wgrad pair (hidden 1024, batch 4000)."""
    from ldnn.models.mlp import mlp3
    from ldnn.train.static_mlp import OptimConfig, StaticMLPEngine

    torch.manual_seed(0)
    B = 4000
    m1, m2 = mlp3(784, 1024, 10), mlp3(784, 1024, 10)
    m2.load_state_dict(m1.state_dict())
    cfg = OptimConfig(opt, lr=0.05 if opt == "sgd" else 1e-3, momentum=0.9)
    e1 = StaticMLPEngine(m1, B, cfg, use_graphs=True)
    e2 = StaticMLPEngine(m2, B, cfg, use_graphs=True, fuse_head_bwd=False)
    assert e1._fuse_head_bwd and not e2._fuse_head_bwd
    g = torch.Generator(device="cuda").manual_seed(5)
    for _ in range(5):
        x = torch.randn(B, 784, device="cuda", generator=g).bfloat16()
        y = torch.randint(0, 10, (B,), device="cuda", generator=g)
        st = []
        for e in (e1, e2):
            e.reset_stats()
            e.load_batch(x, y)
            e.step()
            st.append(e.read_stats(B))
        assert abs(st[0][0] - st[1][0]) < 1e-3 * max(1.0, abs(st[1][0])), st
    atol = 1e-4 if opt == "sgd" else 5 * cfg.lr
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-3, atol=atol)


@pytest.mark.parametrize("B,K,ncls,relu", [(1000, 512, 10, True), (16384, 4096, 10, True), (333, 128, 16, False),
                                           (64, 64, 3, True)])
def test_head_bwd_matches_fp32_and_stream_kernels(B, K, ncls, relu):
    """head_bwd (fused head dgrad + wgrad on MFMA) == fp32 references of dh, its column sums, dW and db,
    and agrees with the head_dgrad_stream + head_wgrad pair it replaces."""
    C = _ext.C()
    g = torch.Generator(device="cuda").manual_seed(7)
    h = torch.randn(B, K, device="cuda", generator=g).bfloat16()
    if relu:
        h = torch.relu(h)
    W = torch.zeros(16, K, device="cuda", dtype=torch.bfloat16)
    W[:ncls] = (torch.randn(ncls, K, device="cuda", generator=g) / K ** 0.5).bfloat16()
    dl = torch.zeros(B, 16, device="cuda", dtype=torch.bfloat16)
    dl[:, :ncls] = (torch.randn(B, ncls, device="cuda", generator=g) / B).bfloat16()
    epi = C.EPI_DRELU if relu else C.EPI_NONE
    dh = torch.full((B, K), float("nan"), device="cuda", dtype=torch.bfloat16)
    dbias = torch.zeros(K, device="cuda")
    dW = torch.zeros(16, K, device="cuda")
    db = torch.zeros(16, device="cuda")
    C.head_bwd(h, W, dl, dh, dW, dbias, epi, db)
    ref = dl.float() @ W.float()
    if relu:
        ref = ref * (h.float() > 0)
    torch.testing.assert_close(dh.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    torch.testing.assert_close(dbias, dh.float().sum(0), rtol=1e-3, atol=1e-3 * dbias.abs().max().item())
    dW_ref = dl.float().t() @ h.float()
    torch.testing.assert_close(dW, dW_ref, rtol=1e-3, atol=1e-3 * dW_ref.abs().max().item())
    torch.testing.assert_close(db, dl.float().sum(0), rtol=1e-3, atol=1e-6)
    # the kernels it replaces
    dh2 = torch.empty_like(dh)
    dbias2 = torch.zeros(K, device="cuda")
    C.head_dgrad_stream(h, W, dl, dh2, dbias2, epi)
    dW2 = torch.zeros(16, K, device="cuda")
    db2 = torch.zeros(16, device="cuda")
    C.head_wgrad(dl, h, dW2, db2, 4)
    diff = (dh.float() - dh2.float()).abs().max().item()
    assert diff <= 1e-2 * ref.abs().max().item(), diff
    torch.testing.assert_close(dW, dW2, rtol=1e-4, atol=1e-4 * dW2.abs().max().item())
