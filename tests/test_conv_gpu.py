"""Implicit-GEMM conv kernels (fwd / dgrad / wgrad) vs PyTorch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

import ldnn
from ldnn.ops import _ext

pytestmark = pytest.mark.gpu

SHAPES = [
    # N, C, H, W, K, R, stride, pad
    (4, 3, 32, 32, 64, 3, 1, 1),      # EnhancedCNN stem (C padded 3 -> 8)
    (4, 64, 32, 32, 128, 3, 2, 1),    # first conv of a stage
    (2, 128, 16, 16, 128, 3, 1, 1),
    (4, 64, 32, 32, 128, 1, 2, 0),    # 1x1 stride-2 shortcut
    (8, 1, 28, 28, 6, 5, 1, 2),       # LeNet conv1 (C 1 -> 8, K 6 -> 8)
    (8, 6, 14, 14, 16, 5, 1, 0),      # LeNet conv2
    (2, 3, 64, 64, 64, 7, 2, 3),      # ResNet stem
]


def up8(v):
    return (v + 7) // 8 * 8


def nhwc(x, cp):
    n, c, h, w = x.shape
    out = torch.zeros(n, h, w, cp, device=x.device, dtype=torch.bfloat16)
    out[..., :c] = x.permute(0, 2, 3, 1)
    return out


def krsc(w, kp, cp):
    k, c, r, s = w.shape
    out = torch.zeros(kp, r, s, cp, device=w.device, dtype=torch.bfloat16)
    out[:k, :, :, :c] = w.permute(0, 2, 3, 1)
    return out


@pytest.mark.parametrize("N,C,H,W,K,R,st,pad", SHAPES)
def test_conv_fwd_dgrad_wgrad(N, C, H, W, K, R, st, pad):
    torch.manual_seed(0)
    Cc = _ext.C()
    x = torch.randn(N, C, H, W, device="cuda").bfloat16().float()
    w = (torch.randn(K, C, R, R, device="cuda") * (1.0 / (C * R * R) ** 0.5)).bfloat16().float()
    cp, kp = up8(C), up8(K)
    P = (H + 2 * pad - R) // st + 1
    xg, wg = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    ref = F.conv2d(xg, wg, None, st, pad)
    gy = torch.randn_like(ref).bfloat16().float()
    ref.backward(gy)

    xn, wn = nhwc(x, cp), krsc(w, kp, cp)
    y = torch.empty(N, P, P, kp, device="cuda", dtype=torch.bfloat16)
    Cc.conv_fwd(xn, wn, y, st, pad)
    out = y[..., :K].permute(0, 3, 1, 2).float()
    torch.testing.assert_close(out, ref.detach(), rtol=2e-2, atol=2e-2 * ref.abs().max().item())

    gyn = nhwc(gy, kp)
    dx = torch.empty(N, H, W, cp, device="cuda", dtype=torch.bfloat16)
    Cc.conv_dgrad(gyn, wn, dx, st, pad)
    got = dx[..., :C].permute(0, 3, 1, 2).float()
    torch.testing.assert_close(got, xg.grad, rtol=2e-2, atol=2e-2 * xg.grad.abs().max().item())
    assert dx[..., C:].abs().max().item() == 0.0 if cp > C else True

    dw = torch.empty(kp, R, R, cp, device="cuda", dtype=torch.float32)
    Cc.conv_wgrad(gyn, xn, dw, st, pad)
    gotw = dw[:K, :, :, :C].permute(0, 3, 1, 2)
    torch.testing.assert_close(gotw, wg.grad, rtol=2e-2, atol=1e-2 * wg.grad.abs().max().item())
