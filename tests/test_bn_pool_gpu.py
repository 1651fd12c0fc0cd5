"""Native NHWC BatchNorm (+residual +ReLU) and pooling vs PyTorch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

import ldnn
from ldnn.models.layers import AdaptiveAvgPool2d, AvgPool2d, BatchNorm2d, MaxPool2d
from ldnn.ops import functional as LF

pytestmark = pytest.mark.gpu


def _cl(x):  # bf16 channels_last copy of a fp32 NCHW tensor
    return x.bfloat16().contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("shape", [(8, 64, 16, 16), (8, 64, 24, 24), (10, 200, 32, 32), (64, 1024, 2, 2),
                                   (16, 40, 4, 4), (17, 64, 64, 64)])
@pytest.mark.parametrize("residual,relu", [(False, False), (False, True), (True, True)])
def test_batchnorm_train_fused(residual, relu, shape):
    """(M = N*H*W <= 2048 rows runs the one-pass small-M statistics kernel; up to 65536 rows the
    same kernel over row groups with per-column tickets (8 x 64 x 24 x 24; 10 x 200 x 32 x 32: a
    partial last column); 17 x 64 x 64 x 64 the multi-block reduce with atomics + last-block
    finalize; C = 40: a partial 64-channel group)"""
    torch.manual_seed(0)
    N, C, H, W = shape
    bn = BatchNorm2d(C)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    ref = torch.nn.BatchNorm2d(C).cuda()
    ref.load_state_dict(bn.state_dict())
    ldnn.prepare(bn, "cuda")
    x = torch.randn(N, C, H, W, device="cuda") * 2 + 0.5
    r = torch.randn(N, C, H, W, device="cuda") if residual else None
    xb = _cl(x).requires_grad_(True)
    rb = _cl(r).requires_grad_(True) if residual else None
    y = bn.act(xb, rb, relu)
    xf = xb.detach().float().requires_grad_(True)
    rf = rb.detach().float().requires_grad_(True) if residual else None
    yr = ref(xf)
    if residual:
        yr = yr + rf
    if relu:
        yr = yr.relu()
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(bn.running_var, ref.running_var, rtol=1e-3, atol=1e-3)
    g = torch.randn_like(yr)
    y.float().backward(g)
    yr.backward(g)
    torch.testing.assert_close(xb.grad.float(), xf.grad, rtol=3e-2, atol=3e-2 * xf.grad.abs().max().item())
    torch.testing.assert_close(bn.weight.grad, ref.weight.grad, rtol=2e-2, atol=2e-2 * ref.weight.grad.abs().max().item())
    torch.testing.assert_close(bn.bias.grad, ref.bias.grad, rtol=2e-2, atol=2e-2 * ref.bias.grad.abs().max().item())
    if residual:
        torch.testing.assert_close(rb.grad.float(), rf.grad, rtol=2e-2, atol=2e-2)


def test_batchnorm_eval_uses_running_stats():
    torch.manual_seed(1)
    C = 32
    bn = BatchNorm2d(C)
    with torch.no_grad():
        bn.running_mean.uniform_(-1, 1)
        bn.running_var.uniform_(0.5, 2)
    ref = torch.nn.BatchNorm2d(C).cuda()
    ref.load_state_dict(bn.state_dict())
    ldnn.prepare(bn, "cuda")
    bn.eval()
    ref.eval()
    x = torch.randn(4, C, 8, 8, device="cuda")
    torch.testing.assert_close(bn(_cl(x)).float(), ref(_cl(x).float()), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("kind,k,st,pad", [("max", 2, 2, 0), ("max", 3, 2, 1), ("avg", 2, 2, 0), ("avg", 3, 1, 1)])
@pytest.mark.parametrize("C", [6, 64])
@pytest.mark.parametrize("flat", [False, True])
def test_pools(kind, k, st, pad, C, flat):
    """(flat: ``flatten_out`` -- the kernel writes a dense NCHW output and its backward reads
    the flattened NCHW gradient, LeNet-5's pool -> fc1 hand-off)"""
    torch.manual_seed(2)
    mod = MaxPool2d(k, st, pad) if kind == "max" else AvgPool2d(k, st, pad)
    mod.flatten_out = flat
    x = torch.randn(4, C, 14, 14, device="cuda")
    xb = _cl(x).requires_grad_(True)
    y = mod(xb)
    if flat:
        assert y.is_contiguous()
        y = y.flatten(1).view(y.shape)
    # reference on a contiguous NCHW copy: torch-ROCm's avg_pool2d backward on a
    # channels_last input returned wrong (asymmetric) gradients for k3/s1/p1 here
    xf = xb.detach().float().contiguous().requires_grad_(True)
    yr = F.max_pool2d(xf, k, st, pad) if kind == "max" else F.avg_pool2d(xf, k, st, pad)
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2)
    g = torch.randn_like(yr).bfloat16().float()
    y.float().backward(g)
    yr.backward(g)
    torch.testing.assert_close(xb.grad.float(), xf.grad, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("shape", [(4, 72, 7, 7), (64, 512, 7, 7), (8, 1024, 4, 4), (2, 64, 2, 2),
                                   (3, 136, 14, 14), (5, 256, 3, 3)])
def test_global_avgpool(shape):
    torch.manual_seed(3)
    x = torch.randn(*shape, device="cuda")
    xb = _cl(x).requires_grad_(True)
    y = AdaptiveAvgPool2d(1)(xb)
    xf = xb.detach().float().requires_grad_(True)
    yr = F.adaptive_avg_pool2d(xf, 1)
    torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2)
    g = torch.randn_like(yr)
    y.float().backward(g)
    yr.backward(g)
    torch.testing.assert_close(xb.grad.float(), xf.grad, rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("residual", [False, True])
def test_bn_relu_mask_matches_reading_y(residual, monkeypatch):
    """BN + ReLU backward from the forward's bit mask == from the bf16 output (bitwise)."""
    torch.manual_seed(1)
    N, C, H, W = 4, 128, 8, 8
    outs = []
    for use_mask in (True, False):
        monkeypatch.setattr(LF, "BN_RELU_MASK", use_mask)
        torch.manual_seed(1)
        bn = BatchNorm2d(C)
        ldnn.prepare(bn, "cuda")
        x = _cl(torch.randn(N, C, H, W, device="cuda")).requires_grad_(True)
        r = _cl(torch.randn(N, C, H, W, device="cuda")).requires_grad_(True) if residual else None
        y = bn.act(x, r, True)
        y.float().backward(torch.linspace(-1, 1, y.numel(), device="cuda").view_as(y))
        outs.append((y.detach().clone(), x.grad.clone(), bn.weight.grad.clone(), bn.bias.grad.clone(),
                     r.grad.clone() if residual else None))
    for a, b in zip(*outs):
        if a is not None:
            torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("op", ["bn_relu", "bn_res_relu", "maxpool", "avgpool"])
def test_twin_output_sums_branch_gradients(op):
    """A native BN / pool output read by two branches through its twin
    (LF.shortcut_input): the producer's backward sums both branch gradients in its
    kernels == the fp32 reference with autograd's accumulation."""
    torch.manual_seed(9)
    N, C, H, W = 8, 64, 18, 18
    x = torch.randn(N, C, H, W, device="cuda") * 1.5 + 0.3
    r = torch.randn(N, C, H, W, device="cuda")
    xb = _cl(x).requires_grad_(True)
    # contiguous NCHW reference (torch-ROCm's channels_last avg_pool2d backward: see test_pools)
    xf = xb.detach().float().contiguous().requires_grad_(True)
    if op.startswith("bn"):
        bn = BatchNorm2d(C)
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
        ref = torch.nn.BatchNorm2d(C).cuda()
        ref.load_state_dict(bn.state_dict())
        ldnn.prepare(bn, "cuda")
        res = op == "bn_res_relu"
        rb = _cl(r) if res else None
        y = bn.act(xb, rb, True)
        yr = (ref(xf) + (rb.float() if res else 0.0)).relu()
    else:
        mod = MaxPool2d(3, 2, 1) if op == "maxpool" else AvgPool2d(3, 2, 1)
        y = mod(xb)
        yr = F.max_pool2d(xf, 3, 2, 1) if op == "maxpool" else F.avg_pool2d(xf, 3, 2, 1)
    twin = LF.shortcut_input(y)
    assert twin is not y and twin.data_ptr() == y.data_ptr()
    g1 = torch.randn_like(yr).bfloat16().float()
    g2 = torch.randn_like(yr).bfloat16().float()
    ((y.float() * g1).sum() + (twin.float() * g2).sum()).backward()
    ((yr * g1).sum() + (yr * g2).sum()).backward()
    torch.testing.assert_close(xb.grad.float(), xf.grad, rtol=3e-2, atol=3e-2 * xf.grad.abs().max().item())


def _stem_pair(C, pad, seed=4):
    torch.manual_seed(seed)
    bn = BatchNorm2d(C)
    with torch.no_grad():
        bn.weight.uniform_(-1.0, 1.5)   # negative gammas too: max(relu(a x + b)) is not a monotone map of x
        bn.bias.uniform_(-0.5, 0.5)
    ref = torch.nn.BatchNorm2d(C).cuda()
    ref.load_state_dict(bn.state_dict())
    ldnn.prepare(bn, "cuda")
    return bn, ref, MaxPool2d(3, 2, pad)


@pytest.mark.parametrize("N,C,H,W,pad", [(4, 64, 20, 18, 1), (2, 16, 11, 13, 1), (3, 32, 12, 12, 0),
                                         (2, 8, 9, 7, 0)])
@pytest.mark.parametrize("twin", [False, True])
def test_bn_relu_maxpool_fused(N, C, H, W, pad, twin, monkeypatch):
    """maxpool3x3/2(relu(BN(x))) in one native pass each way (bn_maxpool_*) == the separate
    native BN-apply + pool pair (identical outputs; gradients up to the fp32 summation order
    of the statistics) and == the fp32 PyTorch reference."""
    x = torch.randn(N, C, H, W, device="cuda") * 2 + 0.3
    g1 = torch.randn(N, C, (H + 2 * pad - 3) // 2 + 1, (W + 2 * pad - 3) // 2 + 1, device="cuda").bfloat16().float()
    g2 = torch.randn_like(g1).bfloat16().float()
    res = []
    for fused in (True, False):
        monkeypatch.setattr(LF, "BN_POOL_FUSED", fused)
        bn, ref, pool = _stem_pair(C, pad)
        xb = _cl(x).requires_grad_(True)
        y = LF.bn_relu_maxpool(xb, bn, pool)
        assert (getattr(y, "_ldnn_twin", None) is not None)
        loss = (y.float() * g1).sum()
        if twin:
            loss = loss + (LF.shortcut_input(y).float() * g2).sum()
        loss.backward()
        res.append((y.detach().float(), xb.grad.float(), bn.weight.grad.clone(), bn.bias.grad.clone(),
                    bn.running_mean.clone(), bn.running_var.clone(), int(bn.num_batches_tracked)))
    (yf, dxf, dgf, dbf, rmf, rvf, nbf), (yu, dxu, dgu, dbu, rmu, rvu, nbu) = res
    assert torch.equal(yf, yu)
    assert nbf == nbu == 1
    torch.testing.assert_close(rmf, rmu, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(rvf, rvu, rtol=1e-5, atol=1e-6)
    # (the separate pool pass rounds the pre-BN gradient to bf16 where windows overlap; the
    # fused pass keeps it fp32)
    torch.testing.assert_close(dgf, dgu, rtol=2e-2, atol=5e-3 * dgu.abs().max().item())
    torch.testing.assert_close(dbf, dbu, rtol=2e-2, atol=5e-3 * dbu.abs().max().item())
    torch.testing.assert_close(dxf, dxu, rtol=2e-2, atol=1e-2 * dxu.abs().max().item())
    # fp32 reference (argmax ties within bf16 rounding may route a gradient to a neighbour:
    # compare dx as a whole)
    bn, ref, pool = _stem_pair(C, pad)
    xf = _cl(x).float().contiguous().requires_grad_(True)
    yr = F.max_pool2d(ref(xf).relu(), 3, 2, pad)
    torch.testing.assert_close(yf, yr, rtol=2e-2, atol=3e-2)
    ((yr * g1).sum() + ((yr * g2).sum() if twin else 0.0)).backward()
    assert ((dxf - xf.grad).norm() / xf.grad.norm()).item() < 3e-2
    assert ((dgf - ref.weight.grad).norm() / ref.weight.grad.norm()).item() < 3e-2
    assert ((dbf - ref.bias.grad).norm() / ref.bias.grad.norm()).item() < 3e-2
    torch.testing.assert_close(rmf, ref.running_mean, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(rvf, ref.running_var, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("N,C,H,W,pad", [(4, 64, 20, 18, 1), (2, 16, 11, 13, 1), (3, 32, 12, 12, 0),
                                         (2, 8, 9, 7, 0), (8, 64, 112, 112, 1)])
@pytest.mark.parametrize("twin", [False, True])
def test_bn_pool_backward_statistics_from_the_pooled_side(N, C, H, W, pad, twin, monkeypatch):
    """LDNN_BN_POOL=1 (default): the forward stores the BN input at every argmax and the backward
    statistics pass sums over pooled positions (dy routed to its argmax, xhat of the stored x)
    instead of reading the whole input; == mode 2 (the pass over x) up to the fp32 summation
    order of the two per-channel sums.  ResNet-18 b256 7.23 -> 7.16 ms
    (profiles/r6/bn_pool_pooled_stats_ab.jsonl)."""
    x = torch.randn(N, C, H, W, device="cuda") * 2 + 0.3
    P, Q = (H + 2 * pad - 3) // 2 + 1, (W + 2 * pad - 3) // 2 + 1
    g1 = torch.randn(N, C, P, Q, device="cuda").bfloat16().float()
    g2 = torch.randn_like(g1).bfloat16().float()
    res = []
    for mode in (1, 2):
        monkeypatch.setattr(LF, "BN_POOL_MODE", mode)
        monkeypatch.setattr(LF, "BN_POOL_FUSED", True)
        bn, ref, pool = _stem_pair(C, pad)
        xb = _cl(x).requires_grad_(True)
        y = LF.bn_relu_maxpool(xb, bn, pool)
        loss = (y.float() * g1).sum()
        if twin:
            loss = loss + (LF.shortcut_input(y).float() * g2).sum()
        loss.backward()
        res.append((y.detach().float(), xb.grad.float(), bn.weight.grad.clone(), bn.bias.grad.clone()))
    (y1, dx1, dg1, db1), (y2, dx2, dg2, db2) = res
    # (above 2048 rows the forward statistics are summed with atomics: both runs' BN outputs may
    # differ in the last bf16 bit, and an argmax tie within one bit may then move)
    assert (y1 != y2).float().mean().item() < 1e-4
    torch.testing.assert_close(y1, y2, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(dg1, dg2, rtol=1e-3, atol=1e-4 * dg2.abs().max().item())
    torch.testing.assert_close(db1, db2, rtol=1e-3, atol=1e-4 * db2.abs().max().item())
    # dx = A g + B x + D: the coefficients differ in the last fp32 bits, dx is rounded to bf16
    assert ((dx1 - dx2).abs() > 1e-2 * dx2.abs().max()).float().mean().item() < 1e-4
    assert ((dx1 - dx2).norm() / dx2.norm()).item() < 2e-3


@pytest.mark.parametrize("N,H", [(16, 112), (16, 224)])
def test_resnet_stem_fused_bn_pool_vs_fp32_oracle(N, H, monkeypatch):
    """ResNet-18's stem -- conv1 7x7/2 (BN statistics from its epilogue) -> bn1 -> ReLU ->
    max-pool 3x3/2 -- with ONE seeded upstream gradient injected at the pool output, in
    three implementations: the fused bn_maxpool pass, the separate BN-apply + pool
    passes, and a plain torch.nn fp32 oracle with the same weights (tests/ref_models.py).

    Why this replaces the round-3 model-level check: at model level the
    gradient reaching the stem is ill-conditioned in ANY bf16 implementation -- stock
    PyTorch-ROCm bf16 autocast differs from fp32 there by 39-42 % and from itself
    run-to-run by 12-14 %, ldnn by 37-40 % / ~20 % (profiles/r4/stem_bn_pool_isolation.txt)
    -- so it cannot separate a kernel bug from rounding.  With the upstream gradient
    fixed the comparison is well conditioned.  Tolerances (bf16 unit roundoff
    u = 2^-9): measured fused-vs-fp32 0.17-0.6 % on dgamma / dbeta, fused-vs-separate
    0.15 %; the conv1 wgrad sits 7.3-7.9 % from fp32 in BOTH paths, and an fp32 oracle
    that only stores the conv output and its gradient in bf16 (what any bf16 pipeline
    stores) sits 6.1-6.7 % from fp32 too: sum(dx * c) = 0 per channel after a BN, so the
    wgrad is a small difference of large terms that amplifies ANY rounding (that oracle
    and ldnn differ from each other by ~6 %, measured).  So dW is pinned by fused ==
    separate (0.22 % apart) and by an error vs fp32 of the same size as the
    bf16-storage oracle's."""
    from ldnn.models import build_model, xavier_init
    from ref_models import oracle_for, rel

    torch.manual_seed(0)
    m = build_model("resnet18")
    xavier_init(m)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    ldnn.prepare(m, "cuda")
    m.train()
    f = m._ldnn_flat
    g = torch.Generator(device="cuda").manual_seed(1234)
    x = torch.randn(N, 3, H, H, device="cuda", generator=g).bfloat16()
    P = ((H + 1) // 2 + 1) // 2
    G = torch.randn(N, 64, P, P, device="cuda", generator=g).bfloat16().float()
    res = {}
    for fused in (True, False):
        monkeypatch.setattr(LF, "BN_POOL_FUSED", fused)
        m.load_state_dict(sd)
        f.refresh_shadow()
        f.reattach_grads()
        f.grad.zero_()
        f._stale.clear()
        y = LF.bn_relu_maxpool(m.conv1(x), m.bn1, m.maxpool)
        (y.float() * G).sum().backward()
        res[fused] = (y.detach().float(), m.bn1.weight.grad.clone(), m.bn1.bias.grad.clone(),
                      m.conv1.weight.grad.clone(), m.bn1.running_mean.clone(), m.bn1.running_var.clone())
    ref = oracle_for("resnet18", sd)
    ref.train()
    xf = x.float()
    yr = ref.stem(xf)
    (yr * G).sum().backward()
    # the bf16-storage oracle: conv output and its gradient rounded to bf16, all math fp32
    emu = oracle_for("resnet18", sd)
    emu.train()
    c = emu.conv1(xf)
    c.register_hook(lambda gr: gr.bfloat16().float())
    cb = c + (c.detach().bfloat16().float() - c.detach())
    (emu.maxpool(torch.relu(emu.bn1(cb))) * G).sum().backward()
    (yf, dgf, dbf, dwf, rmf, rvf), (ys, dgs, dbs, dws, rms, rvs) = res[True], res[False]
    assert rel(yf, ys) < 1e-3                       # same statistics, same bf16 outputs (rare rounding flips)
    assert rel(yf, yr) < 1e-2                       # measured 2.6e-3
    for a, b, what in ((dgf, dgs, "dgamma"), (dbf, dbs, "dbeta"), (dwf, dws, "dW")):
        assert rel(a, b) < 1e-2, (what, rel(a, b))   # fused vs separate: measured <= 2.2e-3
    assert rel(dgf, ref.bn1.weight.grad) < 2e-2, rel(dgf, ref.bn1.weight.grad)   # measured <= 2.3e-3
    assert rel(dbf, ref.bn1.bias.grad) < 3e-2, rel(dbf, ref.bn1.bias.grad)       # measured <= 6.2e-3
    e_emu = rel(emu.conv1.weight.grad, ref.conv1.weight.grad)   # measured 6.1-6.7 %
    assert rel(dwf, ref.conv1.weight.grad) < 2.0 * e_emu + 1e-2, (rel(dwf, ref.conv1.weight.grad), e_emu)
    torch.testing.assert_close(rmf, ref.bn1.running_mean, rtol=1e-2, atol=1e-3 * ref.bn1.running_var.sqrt().max().item())
    torch.testing.assert_close(rvf, ref.bn1.running_var, rtol=1e-2, atol=1e-4)
    torch.testing.assert_close(rmf, rms, rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("N,C,H,W", [(8, 64, 16, 16), (4, 128, 7, 9), (2, 24, 5, 5), (16, 64, 24, 24), (17, 64, 64, 64)])
@pytest.mark.parametrize("twin", [False, True])
@pytest.mark.parametrize("use_mask", [True, False])
def test_bn_dual_act_matches_separate_and_fp32(N, C, H, W, twin, use_mask, monkeypatch):
    """relu(bn_a(x) + bn_b(r)) in one native pass each way (bn_dual_*) == the separate path
    (bn_b's own pass, then bn_a with the residual) and == the fp32 PyTorch reference:
    outputs, running statistics, dx, dr and both BNs' dgamma / dbeta."""
    monkeypatch.setattr(LF, "BN_RELU_MASK", use_mask)
    torch.manual_seed(11)
    x = torch.randn(N, C, H, W, device="cuda") * 1.5 + 0.2
    r = torch.randn(N, C, H, W, device="cuda") * 0.7 - 0.1
    g1 = torch.randn(N, C, H, W, device="cuda").bfloat16().float()
    g2 = torch.randn_like(g1).bfloat16().float()
    res = []
    for fused in (True, False):
        monkeypatch.setattr(LF, "BN_DUAL_FUSED", fused)
        torch.manual_seed(5)
        ba, bb = BatchNorm2d(C), BatchNorm2d(C)
        with torch.no_grad():
            for b in (ba, bb):
                b.weight.uniform_(-1.0, 1.5)
                b.bias.uniform_(-0.5, 0.5)
        refs = [torch.nn.BatchNorm2d(C).cuda() for _ in range(2)]
        refs[0].load_state_dict(ba.state_dict())
        refs[1].load_state_dict(bb.state_dict())
        holder = torch.nn.ModuleList([ba, bb])
        ldnn.prepare(holder, "cuda")
        xb, rb = _cl(x).requires_grad_(True), _cl(r).requires_grad_(True)
        y = LF.batch_norm_dual_act(xb, ba, rb, bb)
        loss = (y.float() * g1).sum()
        if twin:
            loss = loss + (LF.shortcut_input(y).float() * g2).sum()
        loss.backward()
        res.append(dict(y=y.detach().float(), dx=xb.grad.float(), dr=rb.grad.float(),
                        grads=[p.grad.clone() for p in (ba.weight, ba.bias, bb.weight, bb.bias)],
                        stats=[t.clone() for t in (ba.running_mean, ba.running_var, bb.running_mean, bb.running_var)],
                        nb=(int(ba.num_batches_tracked), int(bb.num_batches_tracked)), refs=refs))
    f, u = res
    torch.testing.assert_close(f["y"], u["y"], rtol=1e-2, atol=1e-2)
    assert f["nb"] == u["nb"] == (1, 1)
    for a, b in zip(f["stats"], u["stats"]):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    # gradients as a whole: the separate path rounds bn_b's output to bf16 before the add,
    # the fused pass adds in fp32, so a few ReLU decisions near 0 differ (each moves a
    # channel's sums by one gradient element; measured 1-2 units of sums of ~+-30)
    def rel(a, b):
        return ((a - b).norm() / b.norm()).item()

    for a, b in zip(f["grads"], u["grads"]):
        assert rel(a, b) < 5e-2
    for k in ("dx", "dr"):
        assert rel(f[k], u[k]) < 5e-2
    # fp32 reference
    ra, rb_ = f["refs"]
    xf = _cl(x).float().contiguous().requires_grad_(True)
    rf = _cl(r).float().contiguous().requires_grad_(True)
    yr = (ra(xf) + rb_(rf)).relu()
    torch.testing.assert_close(f["y"], yr, rtol=2e-2, atol=3e-2)
    ((yr * g1).sum() + ((yr * g2).sum() if twin else 0.0)).backward()
    for got, ref in ((f["dx"], xf.grad), (f["dr"], rf.grad)):
        assert rel(got, ref) < 5e-2
    for got, p in zip(f["grads"], (ra.weight, ra.bias, rb_.weight, rb_.bias)):
        assert rel(got, p.grad) < 5e-2
    for got, ref in zip(f["stats"], (ra.running_mean, ra.running_var, rb_.running_mean, rb_.running_var)):
        torch.testing.assert_close(got, ref, rtol=1e-3, atol=1e-3)
