"""Fused pooled classifier head (gap_head.hip: global average pool + Linear in one launch each
way) vs the fp32 PyTorch reference and vs the separate pool + Linear path."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import ldnn
from ldnn.models.layers import AdaptiveAvgPool2d, Linear
from ldnn.ops import functional as LF

pytestmark = pytest.mark.gpu


class _Head(nn.Module):
    def __init__(self, C, ncls):
        super().__init__()
        self.pool = AdaptiveAvgPool2d(1)
        self.fc = Linear(C, ncls)

    def forward(self, x):
        return LF.gap_linear(x, self.pool, self.fc)


def _run(N, C, H, ncls, fused, monkeypatch, steps=1):
    monkeypatch.setattr(LF, "GAP_LINEAR", fused)
    calls = []
    orig = LF._GapLinearNative.apply
    monkeypatch.setattr(LF._GapLinearNative, "apply", lambda *a: calls.append(1) or orig(*a))
    torch.manual_seed(5)
    m = _Head(C, ncls)
    ref = _Head(C, ncls)
    ref.load_state_dict(m.state_dict())
    with torch.no_grad():
        ref.fc.weight.copy_(ref.fc.weight.bfloat16().float())
    ldnn.prepare(m, "cuda")
    x = (torch.randn(N, C, H, H, device="cuda") * 2).bfloat16().contiguous(memory_format=torch.channels_last)
    g = torch.randn(N, ncls, device="cuda")
    xb = x.clone().requires_grad_(True)
    for _ in range(steps):
        y = m(xb)
        y.float().backward(g)
    return m, ref, x, g, y, xb, len(calls)


@pytest.mark.parametrize("N,C,H,ncls", [(64, 1024, 2, 10), (8, 512, 7, 16), (5, 64, 3, 1), (256, 512, 4, 10)])
def test_gap_linear_matches_fp32_and_separate_path(N, C, H, ncls, monkeypatch):
    m, ref, x, g, y, xb, ncalls = _run(N, C, H, ncls, True, monkeypatch)
    assert ncalls == 1, "the fused head did not run"
    xr = x.float().requires_grad_(True)
    ref = ref.cuda()
    yr = F.linear(F.adaptive_avg_pool2d(xr, 1).flatten(1).bfloat16().float(), ref.fc.weight, ref.fc.bias)
    yr.backward(g)
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2 * yr.abs().max().item())
    torch.testing.assert_close(m.fc.weight.grad, ref.fc.weight.grad, rtol=2e-2,
                               atol=1e-2 * ref.fc.weight.grad.abs().max().item())
    torch.testing.assert_close(m.fc.bias.grad, ref.fc.bias.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(xb.grad.float(), xr.grad, rtol=2e-2, atol=1e-2 * xr.grad.abs().max().item())
    # the separate pool + Linear path agrees
    m2, _, _, _, y2, xb2, ncalls2 = _run(N, C, H, ncls, False, monkeypatch)
    assert ncalls2 == 0
    torch.testing.assert_close(y.float(), y2.float(), rtol=1e-2, atol=1e-2 * y2.float().abs().max().item())
    torch.testing.assert_close(m.fc.weight.grad, m2.fc.weight.grad, rtol=1e-2,
                               atol=1e-2 * m2.fc.weight.grad.abs().max().item())
    torch.testing.assert_close(xb.grad.float(), xb2.grad.float(), rtol=1e-2,
                               atol=1e-2 * xb2.grad.float().abs().max().item())


def test_gap_linear_accumulates_gradients(monkeypatch):
    """Two backwards without zeroing: the flat gradient accumulates (grad_beta), as the
    separate path does."""
    m, _, _, _, _, _, _ = _run(16, 256, 2, 10, True, monkeypatch, steps=2)
    m1, _, _, _, _, _, _ = _run(16, 256, 2, 10, True, monkeypatch, steps=1)
    torch.testing.assert_close(m.fc.weight.grad, 2 * m1.fc.weight.grad, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(m.fc.bias.grad, 2 * m1.fc.bias.grad, rtol=1e-5, atol=1e-6)
