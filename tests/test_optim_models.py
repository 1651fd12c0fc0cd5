"""Fused optimizers vs torch.optim; model inventory vs the reference."""
import pytest
import torch

from ldnn.models import build_model, xavier_init
from ldnn.models.mlp import mlp2
from ldnn.optim import SGD, Adam, AdamW, StepLR
from ldnn.utils.flat_params import FlatParams


@pytest.mark.parametrize("Opt,TOpt,kw", [
    (SGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9, weight_decay=1e-4)),
    (SGD, torch.optim.SGD, dict(lr=0.1, momentum=0.9, nesterov=True)),
    (SGD, torch.optim.SGD, dict(lr=0.1)),
    (Adam, torch.optim.Adam, dict(lr=1e-2, weight_decay=1e-3)),
    (AdamW, torch.optim.AdamW, dict(lr=1e-2, weight_decay=1e-2)),
])
@pytest.mark.parametrize("flat", [True, False])
def test_optimizer_matches_torch(Opt, TOpt, kw, flat):
    torch.manual_seed(0)
    m, r = mlp2(784, 32, 10), mlp2(784, 32, 10)
    r.load_state_dict(m.state_dict())
    if flat:
        FlatParams(m, "cpu")
    o, ro = Opt(m.parameters(), **kw), TOpt(r.parameters(), **kw)
    s, rs = StepLR(o, 2, gamma=0.5), StepLR(ro, 2, gamma=0.5)
    for _ in range(5):
        x, y = torch.randn(16, 784), torch.randint(0, 10, (16,))
        for mod, opt in ((m, o), (r, ro)):
            opt.zero_grad()
            torch.nn.functional.cross_entropy(mod(x), y).backward()
            opt.step()
        s.step()
        rs.step()
    for a, b in zip(m.parameters(), r.parameters()):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-6)


def test_optimizer_state_roundtrip():
    torch.manual_seed(0)
    m = mlp2(784, 16, 10)
    FlatParams(m, "cpu")
    o = Adam(m.parameters(), lr=1e-2)
    for _ in range(2):
        o.zero_grad()
        m(torch.randn(4, 784)).sum().backward()
        o.step()
    sd = o.state_dict()
    o2 = Adam(m.parameters(), lr=1e-2)
    o2.load_state_dict(sd)
    assert o2._ls()["step"] == 2
    torch.testing.assert_close(o2._ls()["exp_avg"], o._ls()["exp_avg"])


def test_enhanced_cnn_matches_reference_inventory():
    m = build_model("enhanced_cnn")
    assert sum(p.numel() for p in m.parameters()) == 44_595_786
    assert len(list(m.parameters())) == 65
    sd = m.state_dict()
    assert len(sd) == 128
    for k in ("prep.0.weight", "layer1.0.conv1.weight", "layer1.0.shortcut.0.weight", "layer4.1.bn2.running_var",
              "fc.bias"):
        assert k in sd
    assert sum(p.numel() for p in build_model("enhanced_cnn_small").parameters()) == 4_829_258  # A9
    assert sum(p.numel() for p in build_model("resnet18").parameters()) == 11_689_512


@pytest.mark.parametrize("name,shape", [("enhanced_cnn", (2, 3, 32, 32)), ("lenet5", (2, 1, 28, 28)),
                                        ("mlp3_small", (2, 1, 28, 28)), ("enhanced_cnn_small", (2, 3, 32, 32))])
def test_forward_backward_cpu(name, shape):
    torch.manual_seed(0)
    m = build_model(name)
    xavier_init(m)
    f = FlatParams(m, "cpu")
    out = m(torch.randn(*shape))
    assert out.shape == (2, 10)
    out.sum().backward()
    assert f.grad.abs().sum() > 0
    # every parameter is a view of the flat master, every grad a view of the flat grad buffer
    for p in m.parameters():
        assert p.data_ptr() >= f.master.data_ptr()
        assert p.grad.data_ptr() >= f.grad.data_ptr()


def test_flat_params_padding_stays_zero():
    m = mlp2(784, 20, 10)  # 10-class head -> padded to 16 rows; hidden 20 -> 24
    f = FlatParams(m, "cpu")
    o = SGD(m.parameters(), lr=0.1, momentum=0.9)
    for _ in range(3):
        o.zero_grad()
        torch.nn.functional.cross_entropy(m(torch.randn(8, 784)), torch.randint(0, 10, (8,))).backward()
        o.step()
    w = f.master_storage(m.layers[1].weight)
    assert w.shape == (16, 24)
    assert w[10:].abs().max() == 0 and w[:, 20:].abs().max() == 0


def test_grad_fresh_peeks_without_consuming():
    """FlatParams.grad_fresh reports a lazily zeroed gradient without consuming that state, so the
    dgrad-side BN statistics can check it before the BN's own backward calls grad_beta."""
    m = mlp2(8, 16, 4)
    flat = FlatParams(m)
    w = m[0].weight if hasattr(m, "__getitem__") else next(m.parameters())
    assert flat.grad_beta(w) == 1.0          # nothing marked stale yet: accumulate
    flat.zero_grad(lazy=True)
    assert flat.grad_fresh(w) and flat.grad_fresh(w)   # peeking twice leaves it fresh
    assert flat.grad_beta(w) == 0.0          # the first writer overwrites ...
    assert not flat.grad_fresh(w) and flat.grad_beta(w) == 1.0   # ... and later ones accumulate


@pytest.mark.parametrize("name", ["enhanced_cnn_small", "resnet18"])
def test_downsample_blocks_cpu_match_separate_convs(name):
    """On the CPU (no native launch) LF.conv2d_pair is the two module calls: the downsampling
    blocks that issue their 3x3 and 1x1 convs through it give the plain PyTorch forward."""
    import torch.nn.functional as F

    from ldnn.ops import functional as LF

    torch.manual_seed(0)
    m = build_model(name)
    xavier_init(m)
    blk = next(b for b in m.modules() if getattr(b, "downsample", None) is not None
               or (hasattr(b, "shortcut") and len(getattr(b, "shortcut", [])) > 0))
    conv1 = blk.conv1
    sc = blk.downsample[0] if getattr(blk, "downsample", None) is not None else blk.shortcut[0]
    x = torch.randn(2, conv1.in_channels, 16, 16)
    y0, y1 = LF.conv2d_pair(x, x, conv1, sc)
    torch.testing.assert_close(y0, F.conv2d(x, conv1.weight, conv1.bias, conv1.stride, conv1.padding))
    torch.testing.assert_close(y1, F.conv2d(x, sc.weight, sc.bias, sc.stride, sc.padding))
