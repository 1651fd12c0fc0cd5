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
    (3, 5, 17, 17, 24, 3, 2, 1),      # small-channel VALU dgrad, stride 2
    # LDS-DMA fast path (C / K multiples of 64): 64-channel tiles, ragged rows,
    # stride-2 parity-class dgrad, split-K combine of the small-M tail stages
    (2, 64, 56, 56, 64, 3, 1, 1),     # ResNet layer1 (256x64 tiles)
    (3, 64, 7, 7, 64, 3, 1, 1),       # ragged M (147 rows)
    (2, 128, 15, 15, 256, 3, 2, 1),   # odd H/W stride-2 (uneven parity classes)
    (2, 256, 14, 14, 512, 1, 2, 0),   # 1x1 stride-2 shortcut (empty odd classes)
    (4, 512, 4, 4, 1024, 3, 2, 1),    # EnhancedCNN layer4 first conv (split-K combine)
    (4, 1024, 2, 2, 1024, 3, 1, 1),   # EnhancedCNN tail (split-K combine, huge K)
    (2, 64, 9, 9, 128, 5, 1, 2),      # 5x5 taps on the fast path
    # halo path (3x3 stride 1): channel-block reloads, in-launch split-K, the widest halo
    (2, 256, 14, 14, 256, 3, 1, 1),   # 4 row tiles x 2: split-K slices start mid-block
    (3, 128, 28, 28, 64, 3, 1, 1),    # 256x64 fwd tiles spanning images, 2 channel blocks
    (1, 64, 59, 59, 128, 3, 1, 1),    # W = 59: 2W + 2 = 120 halo rows (the limit)
    (1, 64, 60, 60, 64, 3, 1, 1),     # W = 60: past the halo limit, gather kernel
    # patch path (C = 8 stems, P*Q % 256 == 0): the full ResNet stem, 2 filter tiles, 5x5 taps
    (2, 3, 224, 224, 64, 7, 2, 3),
    (2, 3, 32, 32, 128, 3, 1, 1),
    (2, 8, 32, 32, 64, 5, 1, 2),
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


@pytest.mark.parametrize("N,C,H,W,K,R,st,pad", [(2, 64, 17, 17, 128, 3, 2, 1), (4, 512, 4, 4, 1024, 3, 2, 1),
                                                (2, 128, 16, 16, 64, 3, 1, 1), (4, 1024, 2, 2, 1024, 3, 1, 1),
                                                (2, 8, 40, 40, 64, 7, 2, 3), (3, 16, 9, 9, 32, 3, 1, 1),
                                                (2, 32, 12, 12, 128, 5, 1, 2), (2, 8, 64, 64, 64, 7, 2, 3),
                                                (3, 8, 32, 32, 128, 3, 1, 1), (3, 8, 17, 17, 24, 3, 2, 1),
                                                (4, 8, 14, 14, 16, 5, 1, 0), (3, 8, 13, 13, 16, 3, 1, 1),
                                                (2, 8, 15, 15, 16, 3, 2, 1), (2, 8, 12, 12, 16, 5, 1, 2),
                                                (256, 8, 14, 14, 16, 5, 1, 0), (4, 8, 28, 28, 8, 5, 1, 2), (3, 8, 9, 9, 8, 3, 1, 1)])
def test_lds_fast_path_matches_generic_kernel(N, C, H, W, K, R, st, pad):
    """The LDS-DMA kernels (set_conv_impl(0)) agree with the generic register-staged
    kernels (set_conv_impl(1)) on every output, and repeated launches of the
    split-K combine give bit-identical results (counters reset, order-independent)."""
    torch.manual_seed(1)
    Cc = _ext.C()
    P = (H + 2 * pad - R) // st + 1
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    w = (torch.randn(K, R, R, C, device="cuda") * (1.0 / (C * R * R) ** 0.5)).bfloat16()
    gy = torch.randn(N, P, P, K, device="cuda").bfloat16()
    bias = torch.randn(K, device="cuda")
    outs = {}
    try:
        for impl in (1, 0, 0):
            Cc.set_conv_impl(impl)
            y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
            Cc.conv_fwd(x, w, y, st, pad, bias, Cc.EPI_BIAS_RELU)
            dx = torch.empty(N, H, W, C, device="cuda", dtype=torch.bfloat16)
            Cc.conv_dgrad(gy, w, dx, st, pad)
            dw = torch.randn(K, R, R, C, device="cuda")
            base = dw.clone()
            Cc.conv_wgrad(gy, x, dw, st, pad, 1.0)  # beta = 1 accumulates
            outs.setdefault(impl, []).append((y.float(), dx.float(), dw - base))
    finally:
        Cc.set_conv_impl(0)
    (yg, dxg, dwg), = outs[1]
    (y0, dx0, dw0), (y1, dx1, dw1) = outs[0]
    torch.testing.assert_close(y0, yg, rtol=2e-2, atol=2e-2 * yg.abs().max().item())
    torch.testing.assert_close(dx0, dxg, rtol=2e-2, atol=2e-2 * dxg.abs().max().item())
    torch.testing.assert_close(dw0, dwg, rtol=1e-3, atol=1e-3 * dwg.abs().max().item())
    assert torch.equal(y0, y1) and torch.equal(dx0, dx1)


@pytest.mark.parametrize("dtype,C,cp,H,W", [(torch.float32, 3, 8, 13, 17), (torch.bfloat16, 3, 8, 13, 17),
                                            (torch.float32, 16, 16, 13, 17), (torch.bfloat16, 20, 32, 13, 17),
                                            # H*W % 4 == 0, <= 8 channels: the 4-pixels-per-thread kernel
                                            (torch.float32, 3, 8, 12, 16), (torch.bfloat16, 3, 8, 32, 32),
                                            (torch.bfloat16, 1, 8, 28, 28), (torch.float32, 8, 8, 6, 6)])
def test_nchw_to_nhwc_pad(dtype, C, cp, H, W):
    """Native NCHW -> NHWC bf16 conversion with zeroed pad channels == permute + pad (and the
    labels copied in the same launch)."""
    x = torch.randn(3, C, H, W, device="cuda").to(dtype)
    out = torch.full((3, H, W, cp), 7.0, device="cuda", dtype=torch.bfloat16)
    y = torch.randint(0, 10, (6,), device="cuda")
    ys = torch.full_like(y, -1)
    _ext.C().nchw_to_nhwc(x, out, y, ys)
    ref = torch.zeros(3, H, W, cp, device="cuda", dtype=torch.bfloat16)
    ref[..., :C] = x.permute(0, 2, 3, 1).to(torch.bfloat16)
    assert torch.equal(out, ref)
    assert torch.equal(ys, y)


@pytest.mark.parametrize("N,C,H,W,K", [(2, 64, 56, 56, 64), (2, 128, 28, 28, 128), (3, 256, 14, 14, 256),
                                       (2, 512, 7, 7, 512), (2, 128, 20, 20, 64), (1, 64, 59, 59, 128),
                                       (8, 128, 31, 31, 128), (4, 1024, 2, 2, 1024), (4, 512, 4, 4, 512),
                                       (16, 256, 8, 8, 256), (5, 384, 9, 9, 128)])
def test_halo_conv_matches_gather_kernel(N, C, H, W, K):
    """The halo-staged 3x3 stride-1 kernels == the per-tap gather kernels (set_conv_halo 0),
    bias+ReLU fwd epilogue, split-K slices (in-launch combine and slabs) and channel-block
    reloads included: mode 1 (default: 256x64 tiles) and mode 2 (128x128 tiles too)."""
    torch.manual_seed(3)
    Cc = _ext.C()
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    w = (torch.randn(K, 3, 3, C, device="cuda") * (1.0 / (C * 9) ** 0.5)).bfloat16()
    gy = torch.randn(N, H, W, K, device="cuda").bfloat16()
    bias = torch.randn(K, device="cuda")
    outs = {}
    try:
        for mode in (0, 1, 2):
            Cc.set_conv_halo(mode)
            y = torch.empty(N, H, W, K, device="cuda", dtype=torch.bfloat16)
            Cc.conv_fwd(x, w, y, 1, 1, bias, Cc.EPI_BIAS_RELU)
            dx = torch.empty(N, H, W, C, device="cuda", dtype=torch.bfloat16)
            Cc.conv_dgrad(gy, w, dx, 1, 1)
            outs[mode] = (y.float(), dx.float())
    finally:
        Cc.set_conv_halo(1)
    (y0, dx0) = outs[0]
    for mode in (1, 2):
        y2, dx2 = outs[mode]
        torch.testing.assert_close(y2, y0, rtol=2e-2, atol=2e-2 * y0.abs().max().item())
        torch.testing.assert_close(dx2, dx0, rtol=2e-2, atol=2e-2 * dx0.abs().max().item())


@pytest.mark.parametrize("N", [24, 3])
def test_weight_stationary_stem_matches_patch_kernel_and_fp32(N):
    """The persistent weight-stationary 7x7 / 2 stem (conv_patch_ws_kernel: weights in registers,
    input patches double-buffered a tile ahead; N 24 gives every workgroup several tiles) == the
    per-tile patch kernel (set_conv_ws 0) bit for bit, == the fp32 conv, and its fused BatchNorm
    statistics (kept in registers over a workgroup's tiles) == the patch kernel's."""
    torch.manual_seed(13)
    Cc = _ext.C()
    x = torch.zeros(N, 224, 224, 8, device="cuda", dtype=torch.bfloat16)
    x[..., :3] = torch.randn(N, 224, 224, 3, device="cuda").bfloat16()
    w = torch.zeros(64, 7, 7, 8, device="cuda", dtype=torch.bfloat16)
    w[..., :3] = (torch.randn(64, 7, 7, 3, device="cuda") * 0.08).bfloat16()
    res = {}
    try:
        for m in (0, 1):
            Cc.set_conv_ws(m)
            y = torch.full((N, 112, 112, 64), 7.0, device="cuda", dtype=torch.bfloat16)
            ws = torch.zeros(Cc.bn_workspace_floats(64), device="cuda")
            sm, si = torch.zeros(64, device="cuda"), torch.zeros(64, device="cuda")
            rm, rv = torch.zeros(64, device="cuda"), torch.ones(64, device="cuda")
            Cc.conv_fwd(x, w, y, 2, 3, bn_ws=ws, bn_running_mean=rm, bn_running_var=rv, bn_save_mean=sm,
                        bn_save_invstd=si)
            res[m] = (y, sm, si, rm, rv)
    finally:
        Cc.set_conv_ws(1)
    assert torch.equal(res[1][0], res[0][0])
    for a, b in zip(res[1][1:], res[0][1:]):  # statistics: fp32 sums in another order
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=2,
                                     padding=3).permute(0, 2, 3, 1)
    torch.testing.assert_close(res[1][0].float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    yb = res[1][0].float().reshape(-1, 64)
    torch.testing.assert_close(res[1][1], yb.mean(0), rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(res[1][2], torch.rsqrt(yb.var(0, unbiased=False) + 1e-5), rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("N,H,W", [(64, 56, 56), (2, 56, 56), (3, 9, 11), (1, 63, 63), (5, 5, 5), (24, 28, 28)])
def test_weight_stationary_conv64_matches_halo_and_fp32(N, H, W):
    """The weight-stationary persistent 64 -> 64 channel 3x3 kernels (conv_ws64_kernel: all
    9 taps' weights in registers, one halo per 128-row tile double-buffered a tile ahead) == the
    halo kernel (set_conv_ws 0)
    bit for bit (same MFMA order; to rounding where the halo kernel splits K) for fwd and dgrad,
    and == the fp32 reference.  N 64 at 56 x 56
    gives every workgroup several tiles (the DMA-ahead path); 3 x 9 x 11 a ragged last tile."""
    torch.manual_seed(11)
    Cc = _ext.C()
    x = torch.randn(N, H, W, 64, device="cuda").bfloat16()
    w = (torch.randn(64, 3, 3, 64, device="cuda") * (1.0 / 576 ** 0.5)).bfloat16()
    gy = torch.randn(N, H, W, 64, device="cuda").bfloat16()
    outs, mode = {}, 1
    try:
        for m in (0, mode):
            Cc.set_conv_ws(m)
            y = torch.full((N, H, W, 64), 7.0, device="cuda", dtype=torch.bfloat16)
            Cc.conv_fwd(x, w, y, 1, 1)
            dx = torch.full((N, H, W, 64), 7.0, device="cuda", dtype=torch.bfloat16)
            Cc.conv_dgrad(gy, w, dx, 1, 1)
            outs[m] = (y, dx)
    finally:
        Cc.set_conv_ws(1)
    if N * H * W >= 65536:  # the halo kernel runs unsplit there: same MFMA order, same bits
        assert torch.equal(outs[mode][0], outs[0][0])
        assert torch.equal(outs[mode][1], outs[0][1])
    for a, b in zip(outs[mode], outs[0]):  # small M: the halo kernel splits K (another summation order)
        torch.testing.assert_close(a.float(), b.float(), rtol=1e-2, atol=1e-2 * b.float().abs().max().item())
    xf, wf, gyf = x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), gy.float().permute(0, 3, 1, 2)
    yr = torch.nn.functional.conv2d(xf, wf, padding=1).permute(0, 2, 3, 1)
    dxr = torch.nn.grad.conv2d_input(xf.shape, wf, gyf, padding=1).permute(0, 2, 3, 1)
    torch.testing.assert_close(outs[mode][0].float(), yr, rtol=1e-2, atol=1e-2 * yr.abs().max().item())
    torch.testing.assert_close(outs[mode][1].float(), dxr, rtol=1e-2, atol=1e-2 * dxr.abs().max().item())


@pytest.mark.parametrize("N,H,W", [(16, 16, 16), (3, 9, 11), (2, 8, 8), (64, 56, 56), (8, 28, 28)])
def test_weight_stationary_conv64_takes_the_next_bn_statistics_at_any_m(N, H, W):
    """conv_fwd with the next BN's statistics on the weight-stationary 64 -> 64 kernel: the kernel's
    epilogue computes them (done) == the statistics of its own bf16 output -- also for the small-M
    shapes whose gather-kernel plan is slab split-K (the slab hand-off used to leave them
    uncomputed while reporting done: ResNet-18 at 64 x 64 inputs trained on garbage there)."""
    torch.manual_seed(29)
    Cc = _ext.C()
    x = torch.randn(N, H, W, 64, device="cuda").bfloat16()
    w = (torch.randn(64, 3, 3, 64, device="cuda") * (1.0 / 576 ** 0.5)).bfloat16()
    ws = torch.zeros(Cc.bn_workspace_floats(64), device="cuda")
    for rep in range(2):   # (the second call: the accumulators the first one left clear)
        y = torch.full((N, H, W, 64), 7.0, device="cuda", dtype=torch.bfloat16)
        sm = torch.full((64,), float("nan"), device="cuda")
        si = torch.full((64,), float("nan"), device="cuda")
        done = Cc.conv_fwd(x, w, y, 1, 1, None, 0, bn_ws=ws, bn_gamma=torch.ones(64, device="cuda"),
                           bn_beta=torch.zeros(64, device="cuda"), bn_save_mean=sm, bn_save_invstd=si)
        assert done
        yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2),
                                        padding=1).permute(0, 2, 3, 1)
        torch.testing.assert_close(y.float(), yr, rtol=1e-2, atol=1e-2 * yr.abs().max().item())
        yb = y.float().reshape(-1, 64)
        torch.testing.assert_close(sm, yb.mean(0), rtol=1e-3, atol=1e-4)
        torch.testing.assert_close(si, torch.rsqrt(yb.var(0, unbiased=False) + 1e-5), rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("N,C,H,W,K", [(2, 64, 56, 56, 64), (3, 128, 28, 28, 128), (2, 256, 14, 14, 512),
                                       (4, 512, 7, 7, 512), (5, 64, 9, 9, 128), (2, 128, 16, 16, 256),
                                       (1, 64, 63, 63, 64), (7, 192, 4, 4, 64), (3, 64, 5, 5, 64), (2, 64, 8, 8, 128), (3, 128, 9, 11, 64)])
def test_ring_wgrad_matches_fp32_and_split_k(N, C, H, W, K):
    """The ring wgrad (3x3 stride 1: 64 x 576 blocks, activation rows staged once in an LDS
    ring, edge taps masked) == the fp32 reference and == the split-K gather wgrad, with beta
    0 (slab sum overwrites) and beta 1 (accumulates)."""
    torch.manual_seed(5)
    Cc = _ext.C()
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    gy = torch.randn(N, H, W, K, device="cuda").bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (K, C, 3, 3), gy.float().permute(0, 3, 1, 2),
                                      stride=1, padding=1).permute(0, 2, 3, 1)
    outs = {}
    try:
        for mode in (2, 0):   # 2: the ring wgrad on every eligible shape (default 1: 64 x 64 layers)
            Cc.set_conv_wgrad_ring(mode)
            dw = torch.full((K, 3, 3, C), float("nan"), device="cuda")
            Cc.conv_wgrad(gy, x, dw, 1, 1)
            base = torch.randn(K, 3, 3, C, device="cuda")
            acc = base.clone()
            Cc.conv_wgrad(gy, x, acc, 1, 1, 1.0)
            outs[mode] = (dw, acc - base)
    finally:
        Cc.set_conv_wgrad_ring(1)
    for mode in (2, 0):
        dw, dacc = outs[mode]
        torch.testing.assert_close(dw, ref, rtol=1e-3, atol=1e-3 * ref.abs().max().item())
        torch.testing.assert_close(dacc, ref, rtol=1e-3, atol=2e-3 * ref.abs().max().item())
    torch.testing.assert_close(outs[2][0], outs[0][0], rtol=1e-4, atol=1e-4 * ref.abs().max().item())


@pytest.mark.parametrize("N,Cin,H,W", [(2, 3, 224, 224), (3, 3, 64, 64), (2, 1, 32, 48), (1, 4, 70, 38)])
def test_stem_s2d_wgrad_matches_fp32_and_split_k(N, Cin, H, W):
    """The space-to-depth stem wgrad (7x7 / 2 / pad 3, C padded to 8 with <= 4 data channels,
    real_channels given) == the fp32 reference and == the split-K gather wgrad; beta 0 and 1."""
    torch.manual_seed(9)
    Cc = _ext.C()
    K = 64
    x = torch.zeros(N, H, W, 8, device="cuda", dtype=torch.bfloat16)
    x[..., :Cin] = torch.randn(N, H, W, Cin, device="cuda").bfloat16()
    P, Q = H // 2, W // 2
    gy = torch.randn(N, P, Q, K, device="cuda").bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (K, 8, 7, 7), gy.float().permute(0, 3, 1, 2),
                                      stride=2, padding=3).permute(0, 2, 3, 1)
    outs = {}
    try:
        for mode in (1, 0):
            Cc.set_conv_stem_s2d(mode)
            dw = torch.full((K, 7, 7, 8), float("nan"), device="cuda")
            Cc.conv_wgrad(gy, x, dw, 2, 3, 0.0, real_channels=Cin)
            base = torch.randn(K, 7, 7, 8, device="cuda")
            acc = base.clone()
            Cc.conv_wgrad(gy, x, acc, 2, 3, 1.0, real_channels=Cin)
            outs[mode] = (dw, acc - base)
    finally:
        Cc.set_conv_stem_s2d(1)
    scale = ref.abs().max().item()
    for mode in (1, 0):
        dw, dacc = outs[mode]
        torch.testing.assert_close(dw, ref, rtol=1e-3, atol=1e-3 * scale)
        torch.testing.assert_close(dacc, ref, rtol=1e-3, atol=2e-3 * scale)
    assert (outs[1][0][..., 4:] == 0).all()


@pytest.mark.parametrize("N,Cin,H,W", [(2, 3, 224, 224), (3, 3, 64, 64), (1, 4, 64, 128), (5, 3, 32, 32)])
def test_stem_s2d_forward_matches_fp32_and_its_image_feeds_the_wgrad(N, Cin, H, W):
    """The 7x7 / 2 stem forward on the packed space-to-depth image (conv_fwd(s2d_xs=...),
    conv_s2d_ws_kernel): == the fp32 reference, == the patch kernel up to fp32 summation order,
    the next BN's fused statistics == the output's; the weight gradient on the forward's packed
    image == the one that packs its own (bit for bit)."""
    torch.manual_seed(19)
    Cc = _ext.C()
    K = 64
    assert Cc.stem_s2d_fwd_ok(N, H, W, 8, K, 7, 7, 2, 3, Cin)
    assert not Cc.stem_s2d_fwd_ok(3, 112, 112, 8, K, 7, 7, 2, 3, 3)   # (56 x 56 outputs: not 256-aligned)
    x = torch.zeros(N, H, W, 8, device="cuda", dtype=torch.bfloat16)
    x[..., :Cin] = torch.randn(N, H, W, Cin, device="cuda").bfloat16()
    w = torch.zeros(K, 7, 7, 8, device="cuda", dtype=torch.bfloat16)
    w[..., :Cin] = (torch.randn(K, 7, 7, Cin, device="cuda") * 0.1).bfloat16()
    P, Q = H // 2, W // 2
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), stride=2, padding=3)
    ref = ref.permute(0, 2, 3, 1)
    outs = {}
    for use in (True, False):
        y = torch.empty(N, P, Q, K, device="cuda", dtype=torch.bfloat16)
        xs = torch.empty(N, P + 3, Q + 3, 16, device="cuda", dtype=torch.bfloat16) if use else None
        ws = torch.zeros(Cc.bn_workspace_floats(K), device="cuda")
        sm, si = torch.empty(K, device="cuda"), torch.empty(K, device="cuda")
        done = Cc.conv_fwd(x, w, y, 2, 3, None, 0, bn_ws=ws, bn_gamma=torch.ones(K, device="cuda"),
                           bn_beta=torch.zeros(K, device="cuda"), bn_save_mean=sm, bn_save_invstd=si,
                           real_channels=Cin, s2d_xs=xs)
        assert done
        outs[use] = (y.float(), sm.clone(), si.clone(), xs)
    y1, sm1, si1, xs = outs[True]
    y0 = outs[False][0]
    scale = ref.abs().max().item()
    torch.testing.assert_close(y1, ref, rtol=1e-2, atol=1e-2 * scale)
    torch.testing.assert_close(y1, y0, rtol=1e-2, atol=4e-3 * scale)
    yb = y1.reshape(-1, K)
    torch.testing.assert_close(sm1, yb.mean(0), rtol=1e-3, atol=1e-4 * scale)
    torch.testing.assert_close(1.0 / si1 ** 2, yb.var(0, unbiased=False) + 1e-5, rtol=2e-3, atol=1e-4 * scale ** 2)
    gy = torch.randn(N, P, Q, K, device="cuda").bfloat16()
    d0 = torch.full((K, 7, 7, 8), float("nan"), device="cuda")
    d1 = torch.full((K, 7, 7, 8), float("nan"), device="cuda")
    Cc.conv_wgrad(gy, x, d0, 2, 3, 0.0, real_channels=Cin)
    Cc.conv_wgrad(gy, x, d1, 2, 3, 0.0, real_channels=Cin, s2d_xs=xs)
    assert torch.equal(d0, d1)


def _s2d_reference(x):
    """xs[n][i][j][(dh*2 + dw)*4 + c] = x[n][c][2(i-2) + dh][2(j-2) + dw] (bf16-rounded; zeros outside)."""
    N, C, H, W = x.shape
    Hs, Ws = H // 2 + 3, W // 2 + 3
    pad = torch.zeros(N, C, 2 * Hs, 2 * Ws, device=x.device)
    pad[:, :, 4:4 + H, 4:4 + W] = x.bfloat16().float()
    t = pad.view(N, C, Hs, 2, Ws, 2).permute(0, 2, 4, 3, 5, 1)   # [n][i][j][dh][dw][c]
    ref = torch.zeros(N, Hs, Ws, 2, 2, 4, device=x.device)
    ref[..., :C] = t
    return ref.reshape(N, Hs, Ws, 16).bfloat16()


@pytest.mark.parametrize("N,C,H,W,f32", [(2, 3, 224, 224, True), (3, 3, 30, 40, True), (2, 1, 64, 64, False),
                                         (1, 4, 18, 22, False), (5, 2, 6, 8, True)])
def test_input_staging_writes_the_stem_s2d_image(N, C, H, W, f32):
    """nchw_to_nhwc(..., s2d=img), the graph's input staging ahead of a 7x7 / 2 stem
    (elementwise.hip nchw_to_nhwc_s2d_kernel): its NHWC image == the plain staging's bit for bit,
    the s2d image == the mapping above, the labels ride along; and where the s2d stem forward
    takes the shape, conv_fwd on the staged image (s2d_packed) == conv_fwd packing its own."""
    torch.manual_seed(23)
    Cc = _ext.C()
    x = torch.randn(N, C, H, W, device="cuda")
    x = x if f32 else x.bfloat16()
    lab = torch.randint(0, 10, (16,), device="cuda")
    lab_out = torch.full_like(lab, -1)
    buf0 = torch.full((N, H, W, 8), float("nan"), device="cuda").bfloat16()
    buf1 = torch.full((N, H, W, 8), float("nan"), device="cuda").bfloat16()
    img = torch.full((N, H // 2 + 3, W // 2 + 3, 16), float("nan"), device="cuda").bfloat16()
    Cc.nchw_to_nhwc(x, buf0)
    Cc.nchw_to_nhwc(x, buf1, lab, lab_out, s2d=img)
    torch.cuda.synchronize()
    assert torch.equal(buf0, buf1)
    assert torch.equal(lab, lab_out)
    assert torch.equal(img, _s2d_reference(x.float()))
    if Cc.stem_s2d_fwd_ok(N, H, W, 8, 64, 7, 7, 2, 3, C):
        w = torch.zeros(64, 7, 7, 8, device="cuda", dtype=torch.bfloat16)
        w[..., :C] = (torch.randn(64, 7, 7, C, device="cuda") * 0.1).bfloat16()
        ys = []
        for packed in (False, True):
            y = torch.empty(N, H // 2, W // 2, 64, device="cuda", dtype=torch.bfloat16)
            xs = img if packed else torch.empty_like(img)
            Cc.conv_fwd(buf1, w, y, 2, 3, None, 0, real_channels=C, s2d_xs=xs, s2d_packed=packed)
            ys.append((y, xs))
        assert torch.equal(ys[0][0], ys[1][0])
        assert torch.equal(ys[0][1], img)


@pytest.mark.parametrize("N,C,H,W,K", [(2, 128, 28, 28, 128), (8, 128, 31, 31, 128), (64, 128, 16, 16, 128),
                                       (16, 256, 14, 14, 256), (4, 512, 7, 7, 512), (4, 1024, 2, 2, 1024),
                                       (5, 384, 9, 9, 128), (64, 256, 8, 8, 256), (64, 128, 28, 28, 128),
                                       (3, 128, 14, 14, 256), (2, 256, 12, 12, 128), (2, 128, 33, 33, 128)])
def test_big_tile_halo_conv_matches_gather_and_fp32(N, C, H, W, K):
    """The 8-wave 256x128 halo kernel (conv_hb_kernel: one halo per channel block, the next
    block's halo and 2 weight K-tiles in flight) == the per-tap gather kernel (set_conv_hb 0,
    set_conv_halo 0) and == fp32 for fwd (plain and bias+ReLU) and dgrad, unsplit, in-launch
    split-K combine and slab split-K grids, ragged last tiles and W = 31 (33: past the halo
    limit, the gather kernel runs either way)."""
    torch.manual_seed(17)
    Cc = _ext.C()
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    w = (torch.randn(K, 3, 3, C, device="cuda") * (1.0 / (C * 9) ** 0.5)).bfloat16()
    gy = torch.randn(N, H, W, K, device="cuda").bfloat16()
    bias = torch.randn(K, device="cuda")
    outs = {}
    halo0 = Cc.get_conv_halo()
    try:
        Cc.set_conv_halo(0)
        for mode in (0, 3, 3):   # 3: every eligible shape (the default, 1, takes large dgrad grids only)
            Cc.set_conv_hb(mode)
            y = torch.full((N, H, W, K), 7.0, device="cuda", dtype=torch.bfloat16)
            Cc.conv_fwd(x, w, y, 1, 1)
            yb = torch.full((N, H, W, K), 7.0, device="cuda", dtype=torch.bfloat16)
            Cc.conv_fwd(x, w, yb, 1, 1, bias, Cc.EPI_BIAS_RELU)
            dx = torch.full((N, H, W, C), 7.0, device="cuda", dtype=torch.bfloat16)
            Cc.conv_dgrad(gy, w, dx, 1, 1)
            outs.setdefault(mode, []).append((y.float(), yb.float(), dx.float()))
    finally:
        Cc.set_conv_hb(1)
        Cc.set_conv_halo(halo0)
    ref = outs[0][0]
    outs[1] = outs[3]
    for a, b in zip(outs[1][0], outs[1][1]):   # repeated launches (split-K counters reset): same bits
        assert torch.equal(a, b)
    for a, b in zip(outs[1][0], ref):
        torch.testing.assert_close(a, b, rtol=1e-2, atol=1e-2 * b.abs().max().item())
    xf, wf, gyf = x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), gy.float().permute(0, 3, 1, 2)
    yr = torch.nn.functional.conv2d(xf, wf, padding=1).permute(0, 2, 3, 1)
    dxr = torch.nn.grad.conv2d_input(xf.shape, wf, gyf, padding=1).permute(0, 2, 3, 1)
    y1, yb1, dx1 = outs[1][0]
    torch.testing.assert_close(y1, yr, rtol=1e-2, atol=1e-2 * yr.abs().max().item())
    torch.testing.assert_close(yb1, torch.relu(yr + bias), rtol=1e-2, atol=1e-2 * yr.abs().max().item())
    torch.testing.assert_close(dx1, dxr, rtol=1e-2, atol=1e-2 * dxr.abs().max().item())


@pytest.mark.parametrize("N,C,H,W", [(64, 128, 28, 28), (64, 128, 16, 16), (8, 256, 14, 14)])
def test_big_tile_halo_conv_fused_bn_statistics(N, C, H, W):
    """The next BatchNorm's statistics accumulated in the conv_hb_kernel epilogue (unsplit and
    in-launch split-K grids) == those of the output it stores, as the gather kernel's do."""
    torch.manual_seed(19)
    Cc = _ext.C()
    x = torch.randn(N, H, W, C, device="cuda").bfloat16()
    w = (torch.randn(C, 3, 3, C, device="cuda") * (1.0 / (C * 9) ** 0.5)).bfloat16()
    res = {}
    try:
        for m in (0, 3):
            Cc.set_conv_hb(m)
            y = torch.full((N, H, W, C), 7.0, device="cuda", dtype=torch.bfloat16)
            ws = torch.zeros(Cc.bn_workspace_floats(C), device="cuda")
            sm, si = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
            rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
            used = Cc.conv_fwd(x, w, y, 1, 1, bn_ws=ws, bn_running_mean=rm, bn_running_var=rv, bn_save_mean=sm,
                               bn_save_invstd=si)
            if not used:   # (a slab split-K grid: the BN runs its own statistics pass)
                pytest.skip("fused statistics not taken on this grid")
            res[m] = (y.float(), sm, si, rm, rv)
    finally:
        Cc.set_conv_hb(1)
    res[1] = res[3]
    yb = res[1][0].reshape(-1, C)
    torch.testing.assert_close(res[1][1], yb.mean(0), rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(res[1][2], torch.rsqrt(yb.var(0, unbiased=False) + 1e-5), rtol=1e-3, atol=1e-4)
    for a, b in zip(res[1][1:], res[0][1:]):
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("N,C,H,K", [(64, 512, 4, 512), (64, 1024, 2, 1024), (64, 256, 4, 512), (3, 128, 5, 200)])
def test_slab_split_conv_fused_bn_statistics(N, C, H, K):
    """Slab split-K forward convs (EnhancedCNN's 4x4 / 2x2 tails) followed by a training BN: the
    slab pass (conv_slab_bn_kernel) writes the bf16 output AND finalizes the BN statistics over
    row groups with per-column tickets -- output == fp32 conv, saved mean / invstd == those of the
    stored output, running stats == the EMA, and a repeat (tickets left zero) gives the same bits."""
    torch.manual_seed(23)
    Cc = _ext.C()
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(K, 3, 3, C, device="cuda") * (1.0 / (C * 9) ** 0.5)).bfloat16()
    ws = torch.zeros(Cc.bn_workspace_floats(K), device="cuda")
    nb = torch.zeros(1, dtype=torch.long, device="cuda")
    outs = []
    for _ in range(2):
        y = torch.full((N, H, H, K), 7.0, device="cuda", dtype=torch.bfloat16)
        sm, si = torch.zeros(K, device="cuda"), torch.zeros(K, device="cuda")
        rm, rv = torch.zeros(K, device="cuda"), torch.ones(K, device="cuda")
        used = Cc.conv_fwd(x, w, y, 1, 1, bn_ws=ws, bn_running_mean=rm, bn_running_var=rv, bn_save_mean=sm,
                           bn_save_invstd=si, bn_num_batches=nb)
        assert used
        outs.append((y.float(), sm, si, rm, rv))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)
    assert nb.item() == 2
    y, sm, si, rm, rv = outs[0]
    xf, wf = x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2)
    yr = torch.nn.functional.conv2d(xf, wf, padding=1).permute(0, 2, 3, 1)
    torch.testing.assert_close(y, yr, rtol=1e-2, atol=1e-2 * yr.abs().max().item())
    yb = y.reshape(-1, K)
    mean, var = yb.mean(0), yb.var(0, unbiased=False)
    torch.testing.assert_close(sm, mean, rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(si, torch.rsqrt(var + 1e-5), rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(rm, 0.1 * mean, rtol=1e-3, atol=1e-5)
    torch.testing.assert_close(rv, 0.9 + 0.1 * yb.var(0, unbiased=True), rtol=1e-3, atol=1e-5)


@pytest.mark.parametrize("N,C,H,K,stride", [(64, 128, 16, 128, 1), (64, 256, 8, 256, 1), (64, 128, 16, 256, 2),
                                            (8, 512, 7, 512, 1), (5, 192, 9, 320, 1)])
def test_fixed_summer_split_k_combine_matches_last_arrival(N, C, H, K, stride):
    """In-launch split-K hand-off with the tile's LAST K slice as the summer (it never stores or
    re-reads its own partial) == the last-arrival summer and the fp32 reference, fwd (with the
    next BN's statistics) and dgrad (stride-2: parity classes); repeated launches give the same
    output bits (the counters are left zero)."""
    torch.manual_seed(29)
    Cc = _ext.C()
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(K, 3, 3, C, device="cuda") * (1.0 / (C * 9) ** 0.5)).bfloat16()
    P = (H + 2 - 3) // stride + 1
    gy = torch.randn(N, P, P, K, device="cuda").bfloat16()
    res = {}
    old = Cc.get_conv_combine_last()
    try:
        for mode in (0, 1, 1):
            Cc.set_conv_combine_last(mode)
            y = torch.empty(N, P, P, K, device="cuda", dtype=torch.bfloat16)
            ws = torch.zeros(Cc.bn_workspace_floats(K), device="cuda")
            sm, si = torch.zeros(K, device="cuda"), torch.zeros(K, device="cuda")
            Cc.conv_fwd(x, w, y, stride, 1, bn_ws=ws, bn_save_mean=sm, bn_save_invstd=si)
            dx = torch.empty_like(x)
            Cc.conv_dgrad(gy, w, dx, stride, 1)
            torch.cuda.synchronize()
            res.setdefault(mode, []).append((y.float(), sm, si, dx.float()))
    finally:
        Cc.set_conv_combine_last(old)
    for k in (0, 3):   # fixed summer: the same output bits launch to launch
        assert torch.equal(res[1][0][k], res[1][1][k])
    for k in (1, 2):   # (the BN statistics' fp32 atomics: arrival order)
        torch.testing.assert_close(res[1][0][k], res[1][1][k], rtol=1e-5, atol=1e-6)
    for a, b in zip(res[1][0], res[0][0]):   # vs the last-arrival summer: same sums, another order
        torch.testing.assert_close(a, b, rtol=2e-2, atol=1e-2 * b.abs().max().item())
    xf, wf, gyf = x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), gy.float().permute(0, 3, 1, 2)
    yr = torch.nn.functional.conv2d(xf, wf, stride=stride, padding=1).permute(0, 2, 3, 1)
    dxr = torch.nn.grad.conv2d_input(xf.shape, wf, gyf, stride=stride, padding=1).permute(0, 2, 3, 1)
    y1, sm1, si1, dx1 = res[1][0]
    torch.testing.assert_close(y1, yr, rtol=1e-2, atol=1e-2 * yr.abs().max().item())
    torch.testing.assert_close(dx1, dxr, rtol=1e-2, atol=1e-2 * dxr.abs().max().item())
    yb = y1.reshape(-1, K)
    torch.testing.assert_close(sm1, yb.mean(0), rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("N,C,H,K", [(64, 128, 16, 128), (64, 256, 8, 256), (64, 512, 4, 512), (64, 1024, 2, 1024),
                                     (8, 512, 7, 512), (5, 192, 9, 256),
                                     (64, 64, 56, 64), (16, 64, 32, 64), (3, 64, 9, 64)])
@pytest.mark.parametrize("relu", [True, False])
def test_dgrad_takes_bn_backward_statistics(N, C, H, K, relu):
    """A stride-1 dgrad whose dx is the gradient of a training BN(+ReLU)'s output takes that BN's
    backward statistics (in its slab split-K sum, in one pass over dx right after an unsplit /
    in-launch-combine dgrad, or -- the 64 -> 64 weight-stationary dgrad -- in its persistent
    epilogue, summed per lane over all of a workgroup's tiles) and finalizes them: dx has the bits
    of the plain dgrad, and the BN
    backward's apply pass alone (stats_ready) gives the dx / dgamma / dbeta of the BN's own reduce;
    a repeat (accumulators and tickets left clear) agrees."""
    torch.manual_seed(31)
    _dgrad_bn_stats_case(_ext.C(), N, C, H, K, relu)


def _dgrad_bn_stats_case(Cc, N, C, H, K, relu):
    M = N * H * H
    xb = (torch.randn(M, C, device="cuda") * 1.5 + 0.3).bfloat16()
    gamma = torch.rand(C, device="cuda") + 0.5
    beta = torch.rand(C, device="cuda") - 0.5
    sm, si = torch.empty(C, device="cuda"), torch.empty(C, device="cuda")
    yb = torch.empty_like(xb)
    mask = torch.empty(M * C // 8, dtype=torch.uint8, device="cuda") if relu else None
    Cc.bn_fwd(xb, yb, None, gamma, beta, None, None, sm, si, torch.zeros(Cc.bn_workspace_floats(C), device="cuda"),
              1e-5, 0.0, True, relu, None, mask=mask)
    w = (torch.randn(K, 3, 3, C, device="cuda") * (1.0 / (K * 9) ** 0.5)).bfloat16()
    gy = torch.randn(N, H, H, K, device="cuda").bfloat16()

    def bn_back(dx, ws, ready):
        dg, db = torch.full((C,), 3.0, device="cuda"), torch.full((C,), 3.0, device="cuda")
        out = torch.empty(M, C, device="cuda", dtype=torch.bfloat16)
        if ready:
            used = Cc.conv_dgrad(gy, w, dx, 1, 1, bn_x=xb, bn_mask=mask, bn_ws=ws, bn_gamma=gamma, bn_save_mean=sm,
                                 bn_save_invstd=si, bn_dgamma=dg, bn_dbeta=db, bn_assign=True)
            assert used
        else:
            Cc.conv_dgrad(gy, w, dx, 1, 1)
        Cc.bn_bwd(xb, xb, dx.view(M, C), out, None, gamma, sm, si, ws, dg, db, relu, mask=mask, grad_assign=True,
                  stats_ready=ready)
        torch.cuda.synchronize()
        return dx.float(), out.float(), dg, db

    ws = torch.zeros(Cc.bn_workspace_floats(C), device="cuda")
    ref = bn_back(torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16), torch.zeros_like(ws), False)
    for _ in range(2):
        got = bn_back(torch.empty(N, H, H, C, device="cuda", dtype=torch.bfloat16), ws, True)
        assert torch.equal(got[0], ref[0])
        torch.testing.assert_close(got[2], ref[2], rtol=1e-3, atol=1e-3 * ref[2].abs().max().item())
        torch.testing.assert_close(got[3], ref[3], rtol=1e-3, atol=1e-3 * ref[3].abs().max().item())
        torch.testing.assert_close(got[1], ref[1], rtol=1e-2, atol=1e-2 * ref[1].abs().max().item())
    # the plain statistics left the workspace clear for the fused ones and vice versa
    assert torch.count_nonzero(ws[10 * C + 16: 10 * C + 17]) == 0


@pytest.mark.parametrize("C,H", [(512, 4), (128, 16), (256, 8), (64, 56)])
def test_resblock_bn1_backward_statistics_come_from_conv2_dgrad(C, H):
    """In a residual block, bn1's output feeds conv2 alone: its backward statistics come from
    conv2's dgrad (EnhancedCNN layer3's 512-channel 4x4 block: in the slab split-K sum; the 16x16 /
    8x8 blocks: as a pass over dx in the launch after the shared dgrad + wgrad launch; one fused BN
    backward per step), while the block input -- read by the shortcut through its twin -- keeps the
    BN's own reduce; the gradients match the unfused path."""
    from ldnn.models.cnn import ResBlock
    from ldnn.ops import functional as LF

    torch.manual_seed(37)
    grads = []
    for fused in (False, True):
        torch.manual_seed(37)
        blk = ResBlock(C, C).cuda()
        flat = ldnn.prepare(blk, "cuda")
        x = torch.randn(64, C, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
        old = LF.CONV_BN_BWD
        LF.CONV_BN_BWD = fused
        try:
            for it in range(2):   # step 2: the lazily zeroed gradients (their first writer overwrites)
                flat.zero_grad(lazy=True)
                xi = x.detach().clone().requires_grad_(True)
                n0 = LF.BN_BWD_FUSED[0]
                y = blk(xi)
                y.float().square().sum().backward()
                torch.cuda.synchronize()
            assert LF.BN_BWD_FUSED[0] - n0 == (1 if fused else 0)
        finally:
            LF.CONV_BN_BWD = old
        grads.append([xi.grad.float()] + [p.grad.float().clone() for p in blk.parameters()])
    for a, b in zip(grads[0], grads[1]):
        torch.testing.assert_close(b, a, rtol=2e-2, atol=2e-2 * a.abs().max().item())


@pytest.mark.parametrize("N,C,H,K,stride", [(64, 128, 16, 128, 1), (64, 256, 8, 256, 1), (64, 512, 4, 512, 1),
                                            (64, 1024, 2, 1024, 1), (64, 64, 32, 128, 2), (64, 256, 8, 512, 2),
                                            (64, 64, 56, 64, 1), (16, 64, 32, 64, 1), (5, 192, 9, 320, 1),
                                            (8, 96, 12, 64, 1), (64, 128, 28, 128, 1), (64, 256, 14, 256, 1)])
def test_paired_dgrad_wgrad_launch_matches_separate(N, C, H, K, stride):
    """conv_bwd: a layer's dgrad and wgrad in ONE launch (conv_pair_kernel: the dgrad's workgroups,
    then the wgrad's, each over its own virtual grid) give the bits of the two separate launches
    (split-K slabs / in-launch combine included), for accumulate (beta 1) and overwrite, and match
    the fp32 reference."""
    torch.manual_seed(41)
    Cc = _ext.C()
    P = (H + 2 - 3) // stride + 1
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(K, 3, 3, C, device="cuda") * (1.0 / (K * 9) ** 0.5)).bfloat16()
    gy = torch.randn(N, P, P, K, device="cuda").bfloat16()
    dw0 = torch.randn(K, 3, 3, C, device="cuda")
    old = Cc.get_conv_pair()
    res = []
    try:
        for mode in (0, 1, 1, 2, 3):   # (2 / 3: paired on the generic kernels where a layer alone takes others)
            Cc.set_conv_pair(mode)
            out = []
            for beta in (0.0, 1.0):
                dx = torch.empty_like(x)
                dw = dw0.clone()
                Cc.conv_bwd(gy, w, dx, x, dw, stride, 1, beta)
                torch.cuda.synchronize()
                out += [dx.float(), dw]
            res.append(out)
    finally:
        Cc.set_conv_pair(old)
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)
    for a, b in zip(res[1], res[2]):
        assert torch.equal(a, b)
    xf, wf, gf = x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), gy.float().permute(0, 3, 1, 2)
    dxr = torch.nn.grad.conv2d_input(xf.shape, wf, gf, stride=stride, padding=1).permute(0, 2, 3, 1)
    dwr = torch.nn.grad.conv2d_weight(xf, wf.shape, gf, stride=stride, padding=1).permute(0, 2, 3, 1)
    torch.testing.assert_close(res[1][0], dxr, rtol=2e-2, atol=2e-2 * dxr.abs().max().item())
    torch.testing.assert_close(res[1][1], dwr, rtol=1e-2, atol=1e-2 * dwr.abs().max().item())
    torch.testing.assert_close(res[1][3], dwr + dw0, rtol=1e-2, atol=1e-2 * dwr.abs().max().item())
    for r in res[3:]:
        torch.testing.assert_close(r[0], dxr, rtol=2e-2, atol=2e-2 * dxr.abs().max().item())
        torch.testing.assert_close(r[1], dwr, rtol=1e-2, atol=1e-2 * dwr.abs().max().item())


@pytest.mark.parametrize("cin,cout,H", [(64, 128, 32), (256, 512, 8), (512, 1024, 4), (64, 128, 56)])
def test_downsample_block_convs_share_a_launch(cin, cout, H):
    """A downsampling residual block's 3x3 conv and 1x1 shortcut conv of one input run as ONE
    forward launch (conv_fwd2) -- each with its BN's fused statistics -- and the block's outputs,
    running statistics and gradients equal those of the launches one by one."""
    from ldnn.models.cnn import ResBlock

    Cc = _ext.C()
    old = Cc.get_conv_pair()
    res = []
    try:
        for mode in (0, 1):
            Cc.set_conv_pair(mode)
            torch.manual_seed(43)
            blk = ResBlock(cin, cout, stride=2).cuda()
            flat = ldnn.prepare(blk, "cuda")
            x = torch.randn(16, cin, H, H, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
            for _ in range(2):
                flat.zero_grad(lazy=True)
                xi = x.detach().clone().requires_grad_(True)
                y = blk(xi)
                y.float().square().mean().backward()
            torch.cuda.synchronize()
            res.append([y.float(), xi.grad.float()] + [p.grad.float().clone() for p in blk.parameters()]
                       + [b.float().clone() for b in blk.buffers()])
    finally:
        Cc.set_conv_pair(old)
    for a, b in zip(res[0], res[1]):
        torch.testing.assert_close(b, a, rtol=1e-2, atol=1e-2 * max(a.abs().max().item(), 1e-6))
