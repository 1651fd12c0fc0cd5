"""Autograd-aware ops on the native gfx950 kernels (generic, module-driven path).

Each op has two implementations:
  * GPU: the hand-written HIP kernels (bf16 activations, fp32 accumulation,
    weight gradients written straight into the FlatParams gradient buffer --
    autograd never allocates or accumulates a weight gradient tensor);
  * CPU: the plain PyTorch fp32 reference (used by the orchestration tests and
    as the numerics oracle of the GPU tests).

Reference call sites replaced: nn.Linear + F.relu / sigmoid
(K10, K13; BAR/model.py:68-71,100), nn.CrossEntropyLoss fwd/bwd + argmax
bookkeeping (K14, K15; BAR/trainer.py:207-216).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _ext

ACTS = {"none": None, "relu": 0, "sigmoid": 1}


def _to_bf16(x: torch.Tensor) -> torch.Tensor:
    if x.dtype == torch.bfloat16:
        return x if x.stride(-1) == 1 else x.contiguous()
    return x.to(torch.bfloat16).contiguous()


def _padded_rows_view(g: torch.Tensor, npad: int, zero_pad_guaranteed: bool = True) -> torch.Tensor:
    """[B, N] tensor -> [B, npad] (npad >= N, multiple of 8), copying only if needed.

    A [B, N] view whose row stride is already npad was produced by an ldnn op on
    a padded [B, npad] buffer and is widened in place.  Gradients written by
    ldnn ops have zero padding; forward activations may carry arbitrary (finite)
    values there, which is harmless because the matching weight columns are 0."""
    B, N = g.shape
    if N == npad and g.is_contiguous():
        return g
    if g.stride(1) == 1 and g.stride(0) == npad and g.dtype == torch.bfloat16 and zero_pad_guaranteed:
        return g.as_strided((B, npad), (npad, 1), g.storage_offset())
    out = torch.zeros(B, npad, dtype=torch.bfloat16, device=g.device)
    out[:, :N].copy_(g)
    return out


class _LinearActNative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act, flat):
        C = _ext.C()
        x = _to_bf16(x)
        w = flat.shadow_storage(weight)
        npad, kpad = w.shape
        K = weight.shape[1]
        assert x.shape[-1] == K, f"Linear expects {K} input features, got {x.shape[-1]}"
        x2 = x.reshape(-1, K)
        if kpad != K:
            # pad columns must be 0 so the weight-gradient pad columns stay exactly 0
            # (the producer's pad may hold e.g. sigmoid(0) = 0.5)
            x2 = _padded_rows_view(x2, kpad)
            # through .data: the producer saved this buffer for its own backward and
            # its pad columns never influence that backward (their gradient is 0)
            x2.data[:, K:].zero_()
        y = torch.empty(x2.shape[0], npad, dtype=torch.bfloat16, device=x.device)
        if bias is not None:
            b = flat.master_storage(bias)
        else:
            b = torch.zeros(npad, dtype=torch.float32, device=x.device)
        epi = {None: C.EPI_BIAS, 0: C.EPI_BIAS_RELU, 1: C.EPI_BIAS_SIGMOID}[act]
        C.gemm(x2, w, y, True, True, epi, bias=b)
        ctx.save_for_backward(x2, y)
        ctx.act, ctx.flat, ctx.weight, ctx.bias = act, flat, weight, bias
        ctx.xshape = x.shape
        n = weight.shape[0]
        out = y if n == npad else y[:, :n]
        return out.reshape(*x.shape[:-1], n)

    @staticmethod
    def backward(ctx, gy):
        C = _ext.C()
        x2, y = ctx.saved_tensors
        flat, weight, bias = ctx.flat, ctx.weight, ctx.bias
        npad = y.shape[1]
        g = _padded_rows_view(_to_bf16(gy.reshape(-1, gy.shape[-1])), npad)
        if ctx.act is not None:
            gz = torch.empty_like(y)
            C.act_bwd(g.contiguous(), y, gz, ctx.act)
        else:
            gz = g.contiguous()
        # weight grad straight into the flat fp32 gradient buffer (accumulate)
        C.gemm(gz, x2, flat.grad_storage(weight), False, False, beta=1.0)
        if bias is not None:
            C.colsum(gz, flat.grad_storage(bias), True)
        flat.notify(weight, bias)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(x2.shape, dtype=torch.bfloat16, device=x2.device)
            C.gemm(gz, flat.shadow_storage(weight), dx, True, False)
            K = weight.shape[1]
            if dx.shape[1] != K:
                dx = dx[:, :K]
            dx = dx.reshape(ctx.xshape)
        return dx, None, None, None, None


def linear_act(x, weight, bias=None, act: str = "none", flat=None):
    """y = act(x @ W^T + b); native fused GEMM epilogue on the GPU."""
    a = ACTS[act]
    if _ext.use_native(x):
        if flat is None or flat.shadow is None:
            raise RuntimeError("native Linear needs the model attached to FlatParams (ldnn.prepare(model))")
        return _LinearActNative.apply(x, weight, bias, a, flat)
    y = F.linear(x.float(), weight, bias)
    if a == 0:
        y = F.relu(y)
    elif a == 1:
        y = torch.sigmoid(y)
    return y


class _ActNative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act):
        C = _ext.C()
        xb = _to_bf16(x).contiguous()
        y = torch.empty_like(xb)
        C.act_fwd(xb, y, act)
        ctx.save_for_backward(y)
        ctx.act = act
        ctx.in_dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        g = _to_bf16(gy).contiguous()
        dx = torch.empty_like(y)
        _ext.C().act_bwd(g, y, dx, ctx.act)
        return dx.to(ctx.in_dtype), None


def relu(x):
    if _ext.use_native(x):
        return _ActNative.apply(x, 0)
    return F.relu(x)


def sigmoid(x):
    if _ext.use_native(x):
        return _ActNative.apply(x, 1)
    return torch.sigmoid(x)


class _SoftmaxXentNative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, stats):
        C = _ext.C()
        B, n = logits.shape
        lg = logits if (logits.dtype == torch.bfloat16 and logits.stride(1) == 1) else logits.to(torch.bfloat16).contiguous()
        ld = lg.stride(0)
        dfull = torch.empty(B * ld, dtype=torch.bfloat16, device=lg.device).view(B, ld)
        local = torch.zeros(2, dtype=torch.float32, device=lg.device)
        C.softmax_xent(lg, labels, dfull[:, :n], local, None, n, 1.0 / B)
        if stats is not None:
            stats[:2].add_(local)
        ctx.save_for_backward(dfull)
        ctx.n, ctx.in_dtype = n, logits.dtype
        return local[0] / B

    @staticmethod
    def backward(ctx, go):
        (dfull,) = ctx.saved_tensors
        d = dfull[:, : ctx.n]
        # grad_output is the scalar d(loss); keep the zero padding of the stored rows
        d = (d.float() * go).to(torch.bfloat16) if ctx.in_dtype == torch.bfloat16 else d.float() * go
        if ctx.in_dtype == torch.bfloat16 and dfull.stride(0) != ctx.n:
            full = torch.zeros_like(dfull)
            full[:, : ctx.n] = d
            d = full[:, : ctx.n]
        return d, None, None


def cross_entropy(logits, labels, stats: torch.Tensor | None = None):
    """Mean softmax cross-entropy.  `stats` (device fp32, >= 2) accumulates
    [sum of per-sample loss, #correct] without a host sync."""
    if _ext.use_native(logits):
        return _SoftmaxXentNative.apply(logits, labels, stats)
    lf = logits.float()
    loss = F.cross_entropy(lf, labels)
    if stats is not None:
        with torch.no_grad():
            stats[0] += loss.detach() * labels.numel()
            stats[1] += (lf.argmax(1) == labels).sum()
    return loss


# ------------------------------------------------------------------ conv / BN
def conv2d(x, mod):
    """Convolution of module `mod` (nn.Conv2d parameters).  GPU: bf16 activations,
    fp32 master weights cast in-graph (autograd returns fp32 weight grads into the
    FlatParams buffer).  CPU: fp32 reference."""
    if x.is_cuda and not _ext._DISABLED:
        xb = x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16)
        w = mod.weight.to(torch.bfloat16)
        b = mod.bias.to(torch.bfloat16) if mod.bias is not None else None
        return F.conv2d(xb, w, b, mod.stride, mod.padding, mod.dilation, mod.groups)
    return F.conv2d(x.float(), mod.weight, mod.bias, mod.stride, mod.padding, mod.dilation, mod.groups)


def batch_norm2d(x, mod):
    training = mod.training or not mod.track_running_stats
    mom = 0.0 if mod.momentum is None else mod.momentum
    if mod.training and mod.track_running_stats and mod.num_batches_tracked is not None:
        mod.num_batches_tracked.add_(1)
        if mod.momentum is None:
            mom = 1.0 / float(mod.num_batches_tracked)
    rm = mod.running_mean if (not mod.training or mod.track_running_stats) else None
    rv = mod.running_var if (not mod.training or mod.track_running_stats) else None
    if x.is_cuda and x.dtype == torch.bfloat16:
        y = F.batch_norm(x.float(), rm, rv, mod.weight, mod.bias, training, mom, mod.eps)
        return y.to(torch.bfloat16)
    return F.batch_norm(x.float(), rm, rv, mod.weight, mod.bias, training, mom, mod.eps)
