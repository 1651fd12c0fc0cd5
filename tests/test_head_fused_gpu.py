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
    atol = 1e-4 if opt == "sgd" else 2e-3
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-3, atol=atol)
