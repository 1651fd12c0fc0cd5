"""The BatchNorm-backward statistics fused into the consuming conv's dgrad epilogue
(ops/functional.py BN_BWD_FUSE, conv_lds.hip bnb_stats_epilogue): the gradients of every
parameter equal the separate statistics pass's -- on the reference's EnhancedCNN (each
ResBlock's bn1 -> ReLU -> conv2; stages whose dgrad runs slab split-K fall back), and on a
block whose BN output has a second consumer (the fused sums are then redone from scratch)."""
import pytest
import torch
import torch.nn as nn

import ldnn
from ldnn.models import CrossEntropyLoss, build_model, xavier_init
from ldnn.models.layers import BatchNorm2d, Conv2d
from ldnn.ops import functional as LF

pytestmark = pytest.mark.gpu


def _grads(model, x, y, fuse, monkeypatch):
    monkeypatch.setattr(LF, "BN_BWD_FUSE", fuse)
    for p in model.parameters():
        p.grad = None
    f = model._ldnn_flat
    f.reattach_grads()
    f.grad.zero_()
    f._stale.clear()
    before = LF.BN_BWD_FUSED[0]
    out = model(x)
    loss = CrossEntropyLoss()(out, y)
    loss.backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().float().clone() for n, p in model.named_parameters()}, LF.BN_BWD_FUSED[0] - before


def _close(ga, gb, rtol):
    for k in gb:
        a, b = ga[k], gb[k]
        err = ((a - b).norm() / b.norm().clamp_min(1e-30)).item()
        assert err < rtol, (k, err)


def test_enhanced_cnn_fused_bn_backward_statistics_match(monkeypatch):
    torch.manual_seed(0)
    m = build_model("enhanced_cnn")
    xavier_init(m)
    ldnn.prepare(m, "cuda")
    m.train()
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(64, 3, 32, 32, device="cuda", generator=g).bfloat16()
    y = torch.randint(0, 10, (64,), device="cuda", generator=g)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    g_ref, n0 = _grads(m, x, y, False, monkeypatch)
    m.load_state_dict(sd)   # same BN running statistics / weights
    m._ldnn_flat.refresh_shadow()
    g_fused, n1 = _grads(m, x, y, True, monkeypatch)
    assert n0 == 0 and n1 >= 2, (n0, n1)   # layer1 / layer2 blocks fuse; the slab-split stages fall back
    # same bf16 dx values and the same formulas; only the fp32 summation order differs
    _close(g_fused, g_ref, 2e-3)


class _TwoConsumers(nn.Module):
    """bn -> ReLU output read by a native conv AND by a plain torch op: its gradient is the sum
    of both, so the dgrad's fused statistics (conv part only) must be discarded and redone."""

    def __init__(self):
        super().__init__()
        self.c1 = Conv2d(64, 128, 3, padding=1, bias=False)
        self.bn = BatchNorm2d(128)
        self.c2 = Conv2d(128, 128, 3, padding=1, bias=False)
        self.fc = nn.Linear(128, 10)

    def forward(self, x):
        h = self.bn.act(self.c1(x), relu=True)
        z = self.c2(h).float() + 0.5 * h.float()
        return self.fc(z.mean(dim=(2, 3)))


def test_second_consumer_discards_fused_statistics(monkeypatch):
    torch.manual_seed(0)
    m = _TwoConsumers()
    ldnn.prepare(m, "cuda")
    m.train()
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn(64, 64, 16, 16, device="cuda", generator=g).bfloat16()
    y = torch.randint(0, 10, (64,), device="cuda", generator=g)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    g_ref, _ = _grads(m, x, y, False, monkeypatch)
    m.load_state_dict(sd)
    m._ldnn_flat.refresh_shadow()
    g_fused, n = _grads(m, x, y, True, monkeypatch)
    assert n == 1   # the dgrad fused them ...
    _close(g_fused, g_ref, 2e-3)   # ... and the BN backward redid them: the gradients still match
