"""Numerics of the hand-written gfx950 kernels against plain PyTorch fp32
references of the same op (run on the MI355X box: `pytest -m gpu`)."""
import pytest
import torch

import ldnn
from ldnn.ops import _ext

pytestmark = pytest.mark.gpu


def C():
    return _ext.C()


def _ref_gemm(a, b, a_kc, b_kc):
    A = a.float() if a_kc else a.float().t()
    B = b.float().t() if b_kc else b.float()
    return A @ B


@pytest.mark.parametrize("tile", [128, 256])
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (200, 136, 784), (1000, 264, 72), (64, 16, 4096),
                                   (384, 512, 1000), (520, 776, 520)])
def test_gemm_layouts(tile, a_kc, b_kc, M, N, K):
    torch.manual_seed(0)
    dev = "cuda"
    a = (torch.randn(M, K, device=dev) if a_kc else torch.randn(K, M, device=dev)).bfloat16()
    b = (torch.randn(N, K, device=dev) if b_kc else torch.randn(K, N, device=dev)).bfloat16()
    c = torch.empty(M, N, device=dev, dtype=torch.float32)
    C().gemm(a, b, c, a_kc, b_kc, tile=tile)
    ref = _ref_gemm(a, b, a_kc, b_kc)
    torch.cuda.synchronize()
    err = (c - ref).abs().max().item()
    assert err <= 1e-3 * K ** 0.5 + 1e-3, err
    cb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    C().gemm(a, b, cb, a_kc, b_kc, tile=tile)
    rel = ((cb.float() - ref).abs().max() / ref.abs().max()).item()
    assert rel < 1e-2, rel


@pytest.mark.parametrize("variant", [1, 2, 3])
@pytest.mark.parametrize("a_kc,b_kc", [(True, True), (True, False), (False, False)])
@pytest.mark.parametrize("M,N,K", [(520, 776, 520), (256, 256, 32), (296, 264, 4200)])
def test_gemm256_main_loop_variants(variant, a_kc, b_kc, M, N, K):
    """2-stage BK64 (1) and the 4-/5-slot BK32 LDS rings (2, 3), ragged edges and odd K-step counts."""
    torch.manual_seed(1)
    a = (torch.randn(M, K, device="cuda") if a_kc else torch.randn(K, M, device="cuda")).bfloat16()
    b = (torch.randn(N, K, device="cuda") if b_kc else torch.randn(K, N, device="cuda")).bfloat16()
    ref = _ref_gemm(a, b, a_kc, b_kc)
    c = torch.empty(M, N, device="cuda")
    C().gemm(a, b, c, a_kc, b_kc, tile=256, variant=variant)
    torch.cuda.synchronize()
    assert (c - ref).abs().max().item() <= 1e-3 * K ** 0.5 + 1e-3
    cb = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    C().gemm(a, b, cb, a_kc, b_kc, tile=256, variant=variant)
    assert ((cb.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2


@pytest.mark.parametrize("tile", [128, 256])
def test_gemm_asymmetric_identity(tile):
    """A = I with an asymmetric B catches a transposed C write."""
    n = 256
    a = torch.eye(n, device="cuda").bfloat16()
    b = torch.arange(n * n, device="cuda").reshape(n, n).float().remainder(97).bfloat16()
    c = torch.empty(n, n, device="cuda")
    C().gemm(a, b, c, True, True, tile=tile)  # C = I @ b^T
    assert torch.equal(c, b.float().t())
    C().gemm(a, b, c, True, False, tile=tile)  # C = I @ b
    assert torch.equal(c, b.float())
    C().gemm(a.t().contiguous(), b, c, False, False, tile=tile)  # C = I^T @ b
    assert torch.equal(c, b.float())


@pytest.mark.parametrize("tile", [128, 256])
@pytest.mark.parametrize("epi", ["bias", "relu", "sigmoid"])
def test_gemm_fwd_epilogues(epi, tile):
    torch.manual_seed(1)
    M, N, K = 300, 264, 784
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda")
    y = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    code = {"bias": C().EPI_BIAS, "relu": C().EPI_BIAS_RELU, "sigmoid": C().EPI_BIAS_SIGMOID}[epi]
    C().gemm(x, w, y, True, True, code, bias=bias, tile=tile)
    ref = x.float() @ w.float().t() + bias
    if epi == "relu":
        ref = ref.relu()
    elif epi == "sigmoid":
        ref = ref.sigmoid()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("tile", [128, 256])
@pytest.mark.parametrize("act", ["relu", "sigmoid"])
def test_gemm_dgrad_epilogue_and_dbias(act, tile):
    torch.manual_seed(2)
    M, N, K = 260, 136, 512  # dX[M,K] = dY[M,N] @ W[N,K]
    dy = torch.randn(M, N, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    yprev = torch.randn(M, K, device="cuda")
    yprev = (yprev.relu() if act == "relu" else yprev.sigmoid()).bfloat16()
    dx = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    db = torch.zeros(K, device="cuda")
    code = C().EPI_DRELU if act == "relu" else C().EPI_DSIGMOID
    C().gemm(dy, w, dx, True, False, code, aux=yprev, dbias=db, tile=tile)
    g = dy.float() @ w.float()
    y = yprev.float()
    ref = g * (y > 0) if act == "relu" else g * y * (1 - y)
    torch.testing.assert_close(dx.float(), ref, rtol=2e-2, atol=5e-2)
    torch.testing.assert_close(db, dx.float().sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("tile", [128, 256])
def test_gemm_wgrad_beta_accumulate(tile):
    torch.manual_seed(3)
    B, N, K = 1000, 264, 784  # dW[N,K] = dY^T X
    dy = torch.randn(B, N, device="cuda").bfloat16()
    x = torch.randn(B, K, device="cuda").bfloat16()
    dw = torch.randn(N, K, device="cuda")
    base = dw.clone()
    C().gemm(dy, x, dw, False, False, beta=1.0, tile=tile)
    ref = base + dy.float().t() @ x.float()
    torch.testing.assert_close(dw, ref, rtol=1e-4, atol=1e-2)


def test_softmax_xent_matches_torch():
    torch.manual_seed(4)
    B, Cc, ld = 777, 10, 16
    full = torch.randn(B, ld, device="cuda").bfloat16()
    logits = full[:, :Cc]
    labels = torch.randint(0, Cc, (B,), device="cuda")
    dl = torch.empty(B, ld, device="cuda", dtype=torch.bfloat16)
    stats = torch.zeros(2, device="cuda")
    db = torch.zeros(ld, device="cuda")
    C().softmax_xent(logits, labels, dl[:, :Cc], stats, dbias=db, num_classes=Cc, grad_scale=1.0 / B)
    lf = logits.float().requires_grad_(True)
    loss = torch.nn.functional.cross_entropy(lf, labels)
    loss.backward()
    torch.testing.assert_close(stats[0] / B, loss.detach(), rtol=1e-4, atol=1e-4)
    correct = (lf.detach().argmax(1) == labels).sum().float()
    assert stats[1].item() == correct.item()
    torch.testing.assert_close(dl[:, :Cc].float(), lf.grad, rtol=2e-2, atol=1e-4)
    assert dl[:, Cc:].float().abs().max().item() == 0.0
    torch.testing.assert_close(db[:Cc], dl[:, :Cc].float().sum(0), rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("B,Cc,ld", [(64, 10, 16), (300, 10, 16), (64, 1000, 1000), (5000, 100, 104)])
def test_softmax_xent_finalize(B, Cc, ld):
    """loss_out: the last block writes [mean loss, #correct] and adds the sums into
    stats; its accumulator workspace is left zero (second call sees only its own batch)."""
    torch.manual_seed(7)
    full = torch.randn(B, ld, device="cuda").bfloat16()
    logits = full[:, :Cc]
    labels = torch.randint(0, Cc, (B,), device="cuda")
    dl = torch.empty(B, ld, device="cuda", dtype=torch.bfloat16)
    stats = torch.tensor([1.0, 2.0], device="cuda")
    ref = torch.nn.functional.cross_entropy(logits.float(), labels)
    correct = (logits.float().argmax(1) == labels).sum().item()
    for rep in range(2):
        out = torch.full((2,), -5.0, device="cuda")
        C().softmax_xent(logits, labels, dl[:, :Cc], stats if rep == 0 else None, None, Cc, 1.0 / B,
                         loss_out=out, loss_scale=1.0 / B)
        torch.testing.assert_close(out[0], ref, rtol=1e-4, atol=1e-4)
        assert out[1].item() == correct
    torch.testing.assert_close(stats, torch.tensor([1.0 + ref.item() * B, 2.0 + correct], device="cuda"),
                               rtol=1e-4, atol=1e-3)
    lf = logits.float().requires_grad_(True)
    torch.nn.functional.cross_entropy(lf, labels).backward()
    torch.testing.assert_close(dl[:, :Cc].float(), lf.grad, rtol=2e-2, atol=1e-4)


def test_scale_bf16_and_loss_backward():
    """The native loss backward (grad_output read on the device) == autograd of the fp32 loss."""
    from ldnn.ops import functional as LF

    torch.manual_seed(8)
    x = torch.randn(96, 16, device="cuda").bfloat16()
    src = torch.randn(96, 16, device="cuda").bfloat16()
    out = torch.empty_like(src)
    C().scale_bf16(src, torch.tensor([-2.5], device="cuda"), out)
    torch.testing.assert_close(out.float(), (src.float() * -2.5).bfloat16().float(), rtol=0, atol=0)
    logits = x[:, :10].clone().requires_grad_(True)
    labels = torch.randint(0, 10, (96,), device="cuda")
    (3.0 * LF.cross_entropy(logits, labels)).backward()
    lf = x[:, :10].float().requires_grad_(True)
    (3.0 * torch.nn.functional.cross_entropy(lf, labels)).backward()
    torch.testing.assert_close(logits.grad.float(), lf.grad, rtol=2e-2, atol=2e-4)


def test_sgd_momentum_matches_torch():
    torch.manual_seed(5)
    n = 10_003
    p = torch.randn(n, device="cuda")
    p_ref = p.clone().requires_grad_(True)
    mom = torch.zeros(n, device="cuda")
    sh = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    hp = torch.tensor([0.1, 0.0], device="cuda")
    opt = torch.optim.SGD([p_ref], lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=True)
    for step in range(3):
        g = torch.randn(n, device="cuda")
        C().sgd_step(p, g * 2, mom, sh, hp, 0.5, 0.9, 0.0, 1e-4, True, step == 0)
        p_ref.grad = g.clone()
        opt.step()
    torch.testing.assert_close(p, p_ref.detach(), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(sh.float(), p.bfloat16().float())


def test_adam_matches_torch():
    torch.manual_seed(6)
    n = 4099
    p = torch.randn(n, device="cuda")
    p_ref = p.clone().requires_grad_(True)
    m = torch.zeros(n, device="cuda")
    v = torch.zeros(n, device="cuda")
    hp = torch.tensor([1e-3, 0.0], device="cuda")
    opt = torch.optim.Adam([p_ref], lr=1e-3)
    for _ in range(4):
        g = torch.randn(n, device="cuda")
        C().bump_step(hp)
        C().adam_step(p, g, m, v, None, hp, 1.0, 0.9, 0.999, 1e-8, 0.0, False)
        p_ref.grad = g.clone()
        opt.step()
    torch.testing.assert_close(p, p_ref.detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("two", [False, True])
def test_mix3_with_bf16_neighbour_inputs(two):
    """The gossip exchange's combine: own fp32 gradient + the neighbours' bf16 copies, fp32 out
    (+ the bf16 shadow) == the fp32 formula on the widened inputs."""
    torch.manual_seed(8)
    n = 4099
    x = torch.randn(n, device="cuda")
    y1, y2 = torch.randn(n, device="cuda").bfloat16(), torch.randn(n, device="cuda").bfloat16()
    out = torch.empty_like(x)
    sh = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    C().mix3(out, x, y1, y2 if two else None, 0.4, 0.3, 0.3 if two else 0.0, sh)
    ref = 0.4 * x + 0.3 * y1.float() + (0.3 * y2.float() if two else 0.0)
    torch.testing.assert_close(out, ref, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(sh, ref.bfloat16(), rtol=0, atol=0)


def test_mix3_and_colsum_and_act():
    torch.manual_seed(7)
    n = 5003
    x, y1, y2 = (torch.randn(n, device="cuda") for _ in range(3))
    out = torch.empty_like(x)
    sh = torch.empty(n, device="cuda", dtype=torch.bfloat16)
    C().mix3(out, x, y1, y2, 0.5, 0.25, 0.25, sh)
    torch.testing.assert_close(out, 0.5 * x + 0.25 * y1 + 0.25 * y2)
    xb = torch.randn(333, 72, device="cuda").bfloat16()
    cs = torch.empty(72, device="cuda")
    C().colsum(xb, cs, False)
    torch.testing.assert_close(cs, xb.float().sum(0), rtol=1e-4, atol=1e-3)
    y = torch.empty_like(xb)
    C().act_fwd(xb, y, C().ACT_SIGMOID)
    torch.testing.assert_close(y.float(), xb.float().sigmoid(), rtol=1e-2, atol=1e-2)
    dx = torch.empty_like(xb)
    C().act_bwd(xb, y, dx, C().ACT_SIGMOID)
    yf = y.float()
    torch.testing.assert_close(dx.float(), xb.float() * yf * (1 - yf), rtol=2e-2, atol=1e-2)


@pytest.mark.parametrize("splitk", [2, 5, 8])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_gemm_splitk_wgrad(splitk, beta):
    torch.manual_seed(11)
    B, N, K = 4096, 16, 784  # dW[N,K] = dY^T X, skinny M -> split the batch reduction
    dy = torch.randn(B, N, device="cuda").bfloat16()
    x = torch.randn(B, K, device="cuda").bfloat16()
    dw = torch.randn(N, K, device="cuda")
    base = dw.clone()
    C().gemm(dy, x, dw, False, False, beta=beta, tile=128, splitk=splitk)
    ref = beta * base + dy.float().t() @ x.float()
    torch.testing.assert_close(dw, ref, rtol=1e-4, atol=2e-2)


@pytest.mark.parametrize("N", [10, 16, 40, 64])
@pytest.mark.parametrize("epi", ["none", "bias", "relu"])
def test_gemm_skinny_n_forward(N, epi):
    torch.manual_seed(12)
    M, K = 1000, 4096
    npad = (N + 7) // 8 * 8
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(npad, K, device="cuda") * 0.02).bfloat16()
    bias = torch.randn(npad, device="cuda")
    y = torch.empty(M, npad, device="cuda", dtype=torch.bfloat16)
    code = {"none": C().EPI_NONE, "bias": C().EPI_BIAS, "relu": C().EPI_BIAS_RELU}[epi]
    C().gemm(x, w, y, True, True, code, bias=bias if epi != "none" else None, tile=16)
    ref = x.float() @ w.float().t()
    if epi != "none":
        ref = ref + bias
    if epi == "relu":
        ref = ref.relu()
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("B,K,ncls,ld", [(4096, 4096, 10, 16), (1000, 784, 10, 16), (333, 520, 40, 48)])
def test_head_fwd_xent(B, K, ncls, ld):
    """Fused last Linear + softmax-xent + argmax vs fp32 PyTorch (logits rounded to bf16 first)."""
    torch.manual_seed(2)
    h = torch.randn(B, K, device="cuda").bfloat16()
    W = torch.zeros(ld, K, device="cuda")
    W[:ncls] = torch.randn(ncls, K, device="cuda") * K ** -0.5
    W = W.bfloat16()
    bias = torch.zeros(ld, device="cuda")
    bias[:ncls] = torch.randn(ncls, device="cuda")
    y = torch.randint(0, ncls, (B,), device="cuda")
    logits = torch.empty(B, ld, device="cuda", dtype=torch.bfloat16)
    dl = torch.empty_like(logits)
    stats = torch.zeros((B + 15) // 16, 2, device="cuda")
    C().head_fwd_xent(h, W, bias, y, logits, dl, stats, ncls, 1.0 / B)
    ref = h.float() @ W.float().t() + bias
    assert ((logits.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    assert logits[:, ncls:].float().abs().max().item() == 0.0
    lr = logits.float()[:, :ncls]
    loss = torch.nn.functional.cross_entropy(lr, y, reduction="sum")
    s = stats.sum(0)
    assert abs(s[0].item() - loss.item()) <= 1e-3 * loss.item() + 1e-2
    assert s[1].item() == (lr.argmax(1) == y).sum().item()
    g = (torch.softmax(lr, 1) - torch.nn.functional.one_hot(y, ncls).float()) / B
    assert (dl.float()[:, :ncls] - g).abs().max().item() < 2e-2 / B + 1e-6
    assert dl[:, ncls:].float().abs().max().item() == 0.0


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("epi", ["drelu", "dsigmoid", "none"])
@pytest.mark.parametrize("B,K,ncls,ld", [(4096, 4096, 10, 16), (1000, 784, 10, 16), (70, 520, 10, 16),
                                         (70, 520, 40, 48)])
def test_head_fwd_xent_fused_dgrad(B, K, ncls, ld, epi, mode):
    """The head's dgrad: dh = (dlogits W) * act'(h) plus the previous layer's bias
    gradient (column sums of dh), vs fp32 PyTorch on the kernel's own bf16 dlogits, in
    every dgrad_mode (0 = streaming kernel, 1 = fused re-reading h, 2 = fused from an
    LDS copy of h), incl. a partial last 16-row workgroup (B = 70); the loss path is
    unchanged by the dgrad."""
    if mode == 0 and ld != 16:
        pytest.skip("the streaming dgrad needs ld == 16")
    torch.manual_seed(4)
    h = torch.randn(B, K, device="cuda")
    if epi == "drelu":
        h = h.relu()
    elif epi == "dsigmoid":
        h = h.sigmoid()
    h = h.bfloat16()
    W = torch.zeros(ld, K, device="cuda")
    W[:ncls] = torch.randn(ncls, K, device="cuda") * K ** -0.5
    W = W.bfloat16()
    bias = torch.zeros(ld, device="cuda")
    y = torch.randint(0, ncls, (B,), device="cuda")
    dl, dl2 = (torch.empty(B, ld, device="cuda", dtype=torch.bfloat16) for _ in range(2))
    st, st2 = torch.zeros((B + 15) // 16, 2, device="cuda"), torch.zeros((B + 15) // 16, 2, device="cuda")
    dh = torch.full((B, K), 7.0, device="cuda").bfloat16()
    db = torch.zeros(K, device="cuda")
    cc = C()
    code = {"drelu": cc.EPI_DRELU, "dsigmoid": cc.EPI_DSIGMOID, "none": cc.EPI_NONE}[epi]
    ws = torch.empty(cc.head_dgrad_ws_floats(B, K), device="cuda")
    cc.head_fwd_xent(h, W, bias, y, None, dl, st, ncls, 1.0 / B, dh=dh, dbias=db, dgrad_epi=code, dbias_ws=ws,
                     dgrad_mode=mode)
    cc.head_fwd_xent(h, W, bias, y, None, dl2, st2, ncls, 1.0 / B)
    assert torch.equal(dl, dl2) and torch.equal(st, st2)
    ref = dl.float()[:, :ncls] @ W.float()[:ncls]
    hf = h.float()
    if epi == "drelu":
        ref = ref * (hf > 0)
    elif epi == "dsigmoid":
        ref = ref * hf * (1 - hf)
    scale = ref.abs().max().item()
    assert (dh.float() - ref).abs().max().item() <= 1e-2 * scale
    cs = dh.float().sum(0)
    torch.testing.assert_close(db, cs, rtol=1e-3, atol=1e-4 * cs.abs().max().item())


@pytest.mark.parametrize("splits", [1, 3, 0])
@pytest.mark.parametrize("B,K,ld,rows", [(4096, 4096, 16, 16), (1000, 784, 16, 16), (300, 520, 48, 40)])
def test_head_wgrad(splits, B, K, ld, rows):
    torch.manual_seed(3)
    dz = torch.randn(B, ld, device="cuda")
    dz[:, rows:] = 0
    dz = dz.bfloat16()
    h = torch.randn(B, K, device="cuda").bfloat16()
    dW = torch.zeros(rows, K, device="cuda")
    db = torch.zeros(rows, device="cuda")
    C().head_wgrad(dz, h, dW, db, splits)
    ref = dz.float()[:, :rows].t() @ h.float()
    assert ((dW - ref).abs().max() / ref.abs().max()).item() < 1e-4
    assert (db - dz.float()[:, :rows].sum(0)).abs().max().item() < 1e-2


@pytest.mark.parametrize("splitk", [2, 3, 5])
@pytest.mark.parametrize("case", ["wgrad_f32", "fwd_relu_bf16", "dgrad_dbias_bf16", "wgrad_beta"])
def test_gemm_splitk_inlaunch_combine(splitk, case):
    """128-tile split-K with the in-launch slab combine: any epilogue, deterministic
    (two launches bit-identical: the arrival counters reset themselves)."""
    torch.manual_seed(11)
    M, N, K = 520, 392, 4096
    ws_elems, ncnt = C().gemm_splitk_ws(M, N, splitk)
    ws = torch.empty(ws_elems, device="cuda")
    cnt = torch.zeros(ncnt, device="cuda", dtype=torch.int32)
    if case in ("wgrad_f32", "wgrad_beta"):
        a = torch.randn(K, M, device="cuda").bfloat16()
        b = torch.randn(K, N, device="cuda").bfloat16()
        ref = a.float().t() @ b.float()
        outs = []
        for _ in range(2):
            c = torch.ones(M, N, device="cuda") if case == "wgrad_beta" else torch.empty(M, N, device="cuda")
            C().gemm(a, b, c, False, False, beta=1.0 if case == "wgrad_beta" else 0.0, tile=128, splitk=splitk,
                     ws=ws, cnt=cnt)
            outs.append(c)
        exp = ref + 1.0 if case == "wgrad_beta" else ref
        torch.testing.assert_close(outs[0], exp, rtol=1e-4, atol=1e-3 * K ** 0.5)
    elif case == "fwd_relu_bf16":
        a = torch.randn(M, K, device="cuda").bfloat16()
        b = (torch.randn(N, K, device="cuda") * 0.02).bfloat16()
        bias = torch.randn(N, device="cuda")
        ref = (a.float() @ b.float().t() + bias).relu()
        outs = []
        for _ in range(2):
            c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            C().gemm(a, b, c, True, True, C().EPI_BIAS_RELU, bias=bias, tile=128, splitk=splitk, ws=ws, cnt=cnt)
            outs.append(c)
        torch.testing.assert_close(outs[0].float(), ref, rtol=2e-2, atol=2e-2)
    else:
        dy = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(K, N, device="cuda") * 0.02).bfloat16()
        yprev = torch.randn(M, N, device="cuda").relu().bfloat16()
        outs = []
        for _ in range(2):
            dx = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            db = torch.zeros(N, device="cuda")
            C().gemm(dy, w, dx, True, False, C().EPI_DRELU, aux=yprev, dbias=db, tile=128, splitk=splitk, ws=ws,
                     cnt=cnt)
            outs.append(dx)
        ref = (dy.float() @ w.float()) * (yprev.float() > 0)
        torch.testing.assert_close(outs[0].float(), ref, rtol=2e-2, atol=5e-2)
        torch.testing.assert_close(db, outs[1].float().sum(0), rtol=1e-3, atol=1e-2)
    assert torch.equal(outs[0], outs[1])
    assert int(cnt.abs().sum().item()) == 0


@pytest.mark.parametrize("act", ["relu", "sigmoid"])
@pytest.mark.parametrize("inplace", [False, True])
@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("rows,cols", [(1003, 264), (4096, 512), (7, 8), (200704, 8), (50021, 48)])
def test_act_bwd_colsum_matches_fp32(act, inplace, accumulate, rows, cols):
    """elementwise.hip act_bwd_colsum: dx = act'(y) * dy and out (+)= colsum(dx), vs torch fp32."""
    torch.manual_seed(rows + cols)
    dy = torch.randn(rows, cols, device="cuda").bfloat16()
    pre = torch.randn(rows, cols, device="cuda")
    y = (pre.relu() if act == "relu" else pre.sigmoid()).bfloat16()
    yf, gf = y.float(), dy.float()
    ref_dx = gf * (yf > 0).float() if act == "relu" else gf * yf * (1 - yf)
    base = torch.randn(cols, device="cuda")
    out = base.clone()
    dx = dy.clone() if inplace else torch.empty_like(dy)
    src = dx if inplace else dy
    code = C().ACT_RELU if act == "relu" else C().ACT_SIGMOID
    C().act_bwd_colsum(src, y, dx, out, code, accumulate)
    torch.testing.assert_close(dx.float(), ref_dx, rtol=1e-2, atol=1e-2)
    ref_out = ref_dx.sum(0) + (base if accumulate else 0)
    torch.testing.assert_close(out, ref_out, rtol=1e-3, atol=1e-3 * (rows ** 0.5))



@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("rows,cols", [(200704, 8), (12345, 48), (256, 128), (3, 4096), (40000, 2056), (0, 16)])
def test_colsum_geometries(rows, cols, accumulate):
    """elementwise.hip colsum over narrow (conv-bias) and wide matrices, single-block stores and
    multi-block atomics, vs torch fp32."""
    torch.manual_seed(cols)
    x = torch.randn(rows, cols, device="cuda").bfloat16()
    base = torch.randn(cols, device="cuda")
    out = base.clone()
    C().colsum(x, out, accumulate)
    ref = x.float().sum(0) + (base if accumulate else 0)
    torch.testing.assert_close(out, ref, rtol=1e-3, atol=1e-3 * max(1.0, rows ** 0.5))


@pytest.mark.parametrize("rows,cols", [(200704, 8), (25600, 16), (12345, 48), (40000, 2056), (256, 128), (0, 16)])
def test_colsum_with_ticketed_scratch_is_one_launch_and_leaves_it_clean(rows, cols):
    """colsum / act_bwd_colsum with ws (the conv bias path): the overwriting multi-group sum runs
    through the caller's zeroed scratch and a ticket instead of a zero fill + atomics into out --
    == torch fp32, and ws (sums and ticket) is zero again after each call, so back-to-back calls
    (a graph replay) give the same result."""
    torch.manual_seed(rows + 7 * cols)
    x = torch.randn(rows, cols, device="cuda").bfloat16()
    ws = torch.zeros(cols + 1, device="cuda")
    ref = x.float().sum(0)
    for _ in range(2):
        out = torch.full((cols,), float("nan"), device="cuda")
        C().colsum(x, out, False, ws=ws)
        torch.testing.assert_close(out, ref, rtol=1e-3, atol=1e-3 * max(1.0, rows ** 0.5))
        assert int((ws != 0).sum().item()) == 0
    y = torch.randn(rows, cols, device="cuda").relu().bfloat16()
    dx = torch.empty_like(x)
    ref_dx = x.float() * (y.float() > 0).float()
    for _ in range(2):
        out = torch.full((cols,), float("nan"), device="cuda")
        C().act_bwd_colsum(x, y, dx, out, C().ACT_RELU, False, ws=ws)
        torch.testing.assert_close(dx.float(), ref_dx, rtol=1e-2, atol=1e-2)
        torch.testing.assert_close(out, ref_dx.sum(0), rtol=1e-3, atol=1e-3 * max(1.0, rows ** 0.5))
        assert int((ws != 0).sum().item()) == 0
