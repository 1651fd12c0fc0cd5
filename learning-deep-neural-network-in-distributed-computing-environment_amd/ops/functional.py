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

import os

import torch
import torch.nn.functional as F

from . import _ext

ACTS = {"none": None, "relu": 0, "sigmoid": 1}


def _fire_pre_hooks(mods, x) -> bool:
    """A fused launch that stands in for the __call__ of several modules (conv2d_pair,
    gap_linear) must still run their forward pre-hooks: the sharded DP step cuts its graph
    chain there and waits for the bucket's weight all-gather (GraphedDPStep._on_forward).
    Fires every module's pre-hooks with (x,) and returns True, or returns False without
    firing any when a module carries hooks a fused launch cannot honour (post-forward
    hooks, kwargs pre-hooks, global module hooks): the caller then runs the module calls."""
    from torch.nn.modules import module as _m

    if _m._global_forward_pre_hooks or _m._global_forward_hooks:
        return False
    for mod in mods:
        if mod._forward_hooks or getattr(mod, "_forward_pre_hooks_with_kwargs", None):
            return False
    for mod in mods:
        for hook in tuple(mod._forward_pre_hooks.values()):
            if hook(mod, (x,)) is not None:
                raise RuntimeError(f"a forward pre-hook of {type(mod).__name__} rewrote its input: "
                                   "not supported on the fused launch")
    return True


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
            zp = getattr(x, "_ldnn_zpad", False)
            x2 = _padded_rows_view(x2, kpad)
            if not zp:
                # through .data: the producer saved this buffer for its own backward and
                # its pad columns never influence that backward (their gradient is 0)
                x2.data[:, K:].zero_()
        y = torch.empty(x2.shape[0], npad, dtype=torch.bfloat16, device=x.device)
        if bias is not None:
            b = flat.master_storage(bias)
        else:
            b = torch.zeros(npad, dtype=torch.float32, device=x.device)
        epi = {None: C.EPI_BIAS, 0: C.EPI_BIAS_RELU, 1: C.EPI_BIAS_SIGMOID}[act]
        # (a split-K forward with the in-launch combine for the 64 x 512 -> 1000 classifier
        # measured slower standalone and neutral in the ResNet-18 step: removed in round 4,
        # profiles/r3s3/head_micro.jsonl)
        C.gemm(x2, w, y, True, True, epi, bias=b)
        ctx.save_for_backward(x2, y)
        ctx.act, ctx.flat, ctx.weight, ctx.bias = act, flat, weight, bias
        ctx.xshape = x.shape
        n = weight.shape[0]
        out = y if n == npad else y[:, :n]
        out = out.reshape(*x.shape[:-1], n)
        if act != 1 and n != npad and out.dim() == 2:
            # pad rows of W and pad entries of b are exactly 0 (their gradients are), so the
            # pad columns hold act(0) = 0: a padded consumer skips re-zeroing them
            out._ldnn_zpad = True
        return out

    @staticmethod
    def backward(ctx, gy):
        C = _ext.C()
        x2, y = ctx.saved_tensors
        flat, weight, bias = ctx.flat, ctx.weight, ctx.bias
        npad = y.shape[1]
        g = _padded_rows_view(_to_bf16(gy.reshape(-1, gy.shape[-1])), npad)
        if ctx.act is not None:
            gz = torch.empty_like(y)
            if bias is not None:   # activation backward + the bias gradient's column sums in one pass
                C.act_bwd_colsum(g.contiguous(), y, gz, flat.grad_storage(bias), ctx.act,
                                 flat.grad_beta(bias) != 0.0)
            else:
                C.act_bwd(g.contiguous(), y, gz, ctx.act)
        else:
            gz = g.contiguous()
            if bias is not None:
                C.colsum(gz, flat.grad_storage(bias), flat.grad_beta(bias) != 0.0)
        # weight grad straight into the flat fp32 gradient buffer (accumulate, or
        # overwrite as the step's first write: FlatParams.grad_beta)
        C.gemm(gz, x2, flat.grad_storage(weight), False, False, beta=flat.grad_beta(weight))
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


def _flat_dense(t: torch.Tensor) -> torch.Tensor | None:
    """A 1-D view over the storage of a dense tensor (row-major or channels_last)."""
    if t.is_contiguous():
        return t.view(-1)
    if t.dim() == 4 and t.is_contiguous(memory_format=torch.channels_last):
        return t.permute(0, 2, 3, 1).reshape(-1)
    return None


class _ActNative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act):
        C = _ext.C()
        xb = x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16)
        if _flat_dense(xb) is None:
            xb = xb.contiguous()
        y = torch.empty_like(xb)  # keeps the memory format (channels_last stays NHWC)
        C.act_fwd(_flat_dense(xb), _flat_dense(y), act)
        ctx.save_for_backward(y)
        ctx.act = act
        ctx.in_dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        g = gy if gy.dtype == torch.bfloat16 else gy.to(torch.bfloat16)
        if g.stride() != y.stride():
            g = g.contiguous(memory_format=torch.channels_last) if y.dim() == 4 and not y.is_contiguous() \
                else g.contiguous()
        dx = torch.empty_like(y)
        _ext.C().act_bwd(_flat_dense(g), _flat_dense(y), _flat_dense(dx), ctx.act)
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
        # one launch: the kernel's last block writes [mean loss, #correct] into `out`
        # and adds [loss sum, #correct] into `stats` (no fill / divide / add kernels)
        out = torch.empty(2, dtype=torch.float32, device=lg.device)
        C.softmax_xent(lg, labels, dfull[:, :n], stats, None, n, 1.0 / B, loss_out=out, loss_scale=1.0 / B)
        ctx.save_for_backward(dfull)
        ctx.n, ctx.in_dtype = n, logits.dtype
        return out[0]

    @staticmethod
    def backward(ctx, go):
        (dfull,) = ctx.saved_tensors
        if ctx.in_dtype == torch.bfloat16 and getattr(go, "_ldnn_unit", False):
            # the graphed steps' persistent seed is exactly 1 (train.graphed.unit_seed): the
            # forward's d(mean loss)/d(logits) is the gradient as is, no scaling pass
            return dfull[:, : ctx.n], None, None
        if ctx.in_dtype == torch.bfloat16 and go.dtype == torch.float32 and go.is_cuda and dfull.numel() % 8 == 0:
            # d = dlogits * grad_output in one pass over the padded rows (pad stays 0)
            full = torch.empty_like(dfull)
            _ext.C().scale_bf16(dfull, go.reshape(1), full)
            return full[:, : ctx.n], None, None
        d = dfull[:, : ctx.n]
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
def _up8(v: int) -> int:
    return (v + 7) // 8 * 8


def as_nhwc(t: torch.Tensor, cp: int, zero_pad: bool = True) -> torch.Tensor:
    """Logical [N, C, H, W] tensor -> dense NHWC bf16 buffer [N, H, W, cp].

    Channels-last tensors (ours, or torch's channels_last outputs) are widened
    in place when their channel stride already is cp; anything else is copied
    into a zero-padded buffer."""
    N, C, H, W = t.shape
    if (t.dtype == torch.bfloat16 and t.stride(1) == 1 and t.stride(3) == cp and t.stride(2) == W * cp
            and t.stride(0) == H * W * cp):
        buf = t.as_strided((N, H, W, cp), (H * W * cp, W * cp, cp, 1), t.storage_offset())
        if zero_pad and cp > C and not getattr(t, "_ldnn_zpad", False):
            buf.data[..., C:].zero_()
        return buf
    if (cp % 8 == 0 and t.is_contiguous() and t.dtype in (torch.float32, torch.bfloat16)
            and _ext.use_native(t)):
        # one native pass: gather + cast + zeroed pad channels (no fill + permute copy)
        buf = torch.empty(N, H, W, cp, dtype=torch.bfloat16, device=t.device)
        _ext.C().nchw_to_nhwc(t, buf)
        return buf
    buf = torch.zeros(N, H, W, cp, dtype=torch.bfloat16, device=t.device) if cp > C else \
        torch.empty(N, H, W, cp, dtype=torch.bfloat16, device=t.device)
    buf[..., :C].copy_(t.permute(0, 2, 3, 1))
    return buf


def nchw_view(buf: torch.Tensor, c: int) -> torch.Tensor:
    """Dense NHWC buffer -> logical [N, c, H, W] view (channels_last strides)."""
    return buf[..., :c].permute(0, 3, 1, 2)


def _zpad(t: torch.Tensor) -> torch.Tensor:
    """Mark a native op's NHWC output whose pad channels (c .. cp-1) are exactly zero by
    construction (zero weight rows / bias entries, pooling or gradients of zero pads), so
    its consumer's as_nhwc skips the pad-clearing launch."""
    t._ldnn_zpad = True
    return t


def _bn_train_state(mod, dev):
    """(running_mean, running_var, momentum, num_batches tensor) of a training-mode BN
    forward, with the Python-side bookkeeping of one call (num_batches_tracked)."""
    mom = mod.momentum
    nbt = None
    if mod.training and mod.track_running_stats:
        # num_batches_tracked += 1 happens inside the fused BN statistics kernel
        nbt = mod.num_batches_tracked if mod.num_batches_tracked.is_cuda else None
        if nbt is None:
            mod.num_batches_tracked.add_(1)
        mod._ldnn_nbt = getattr(mod, "_ldnn_nbt", 0) + 1
        if mom is None:
            mom = 1.0 / mod._ldnn_nbt
    rm = mod.running_mean if mod.track_running_stats else None
    rv = mod.running_var if mod.track_running_stats else None
    return rm, rv, mom, nbt


def _fused_bn_ok(bn, K: int, kp: int, bias, relu: bool) -> bool:
    return (bn is not None and bn.training and bn.affine and kp == K == bn.num_features and bias is None
            and not relu and getattr(bn, "_ldnn_flat", None) is not None)


# The dgrad of a conv whose input is a training BatchNorm(+ReLU)'s output takes that BN's
# backward statistics in its epilogue (conv2d_dgrad with a BnBwdFuse), and the BN backward runs
# its apply pass alone -- one reduce launch less per such pair (LDNN_CONV_BN_BWD=0: off)
CONV_BN_BWD = os.environ.get("LDNN_CONV_BN_BWD", "1") != "0"
BN_BWD_FUSED = [0]   # BN backwards that found their statistics finalized by a dgrad (tests)


class _BnBwdSrc:
    """What a consumer conv's dgrad needs to take a BN's backward statistics (attached to the
    BN's primary output as ``_ldnn_bnsrc``).  ``twin_used``: the output also feeds a shortcut
    (its gradient arrives in two parts, so only the BN's own reduce sees the sum)."""

    __slots__ = ("mod", "flat", "weight", "bias", "x2", "mask", "smean", "sinv", "ws", "C", "twin_used", "pre")

    def __init__(self, mod, flat, weight, bias, x2, mask, smean, sinv, ws, C):
        self.mod, self.flat, self.weight, self.bias = mod, flat, weight, bias
        self.x2, self.mask, self.smean, self.sinv, self.ws, self.C = x2, mask, smean, sinv, ws, C
        self.twin_used = False
        self.pre = None   # (dx pointer, version) of a dgrad that finalized the statistics

    def dgrad_kwargs(self):
        """conv_dgrad keyword arguments, or None when the BN's gradients accumulate this step
        (the fused finalize only overwrites: a recomputing fallback must be able to redo it)."""
        f = self.flat
        if not (f.grad_fresh(self.weight) and f.grad_fresh(self.bias)):   # (peeks: the BN's backward consumes)
            return None
        C = self.C
        return dict(bn_x=self.x2, bn_mask=self.mask, bn_ws=self.ws, bn_gamma=f.master_storage(self.weight)[:C],
                    bn_save_mean=self.smean, bn_save_invstd=self.sinv, bn_dgamma=f.grad_storage(self.weight)[:C],
                    bn_dbeta=f.grad_storage(self.bias)[:C], bn_assign=True)


def _conv_bn_stats(bn, K: int, dev, C):
    """(conv_fwd's bn_* arguments without the prefix, bookkeeping state) for a conv whose epilogue
    takes the next training BN's statistics (_fused_bn_ok)."""
    ws = _bn_workspace(bn, K, dev, C)
    smean = torch.empty(K, dtype=torch.float32, device=dev)
    sinv = torch.empty(K, dtype=torch.float32, device=dev)
    bflat = bn._ldnn_flat
    snap = (getattr(bn, "_ldnn_nbt", 0), bn.num_batches_tracked.clone()
            if bn.track_running_stats and not bn.num_batches_tracked.is_cuda else None)
    rm, rv, mom, nbt = _bn_train_state(bn, dev)
    args = dict(ws=ws, gamma=bflat.master_storage(bn.weight)[:K], beta=bflat.master_storage(bn.bias)[:K],
                running_mean=rm, running_var=rv, save_mean=smean, save_invstd=sinv, eps=bn.eps,
                momentum=mom or 0.0, num_batches=nbt)
    return args, (smean, sinv, snap)


def _conv_bn_stats_done(bn, done: bool, y, state):
    smean, sinv, snap = state
    if done:
        bn.__dict__["_ldnn_pre"] = (y.data_ptr(), smean, sinv)
    else:  # generic conv path: the BN runs its own statistics pass (undo the bookkeeping)
        bn._ldnn_nbt = snap[0]
        if snap[1] is not None:
            bn.num_batches_tracked.copy_(snap[1])


def _colsum_ws(flat, bias, cols: int, dev) -> torch.Tensor:
    """A conv bias's persistent colsum scratch (cols floats + a ticket, zeroed once; the kernel leaves it
    zero): its column sums over many row groups then take one launch, no zero fill (elementwise.hip)."""
    cache = flat.__dict__.setdefault("_ldnn_colsum_ws", {})
    ws = cache.get(id(bias))
    if ws is None or ws.device != dev or ws.numel() < cols + 1:
        ws = torch.zeros(cols + 1, dtype=torch.float32, device=dev)
        cache[id(bias)] = ws
    return ws


class _Conv2dNative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad, flat, relu, bn=None):
        C = _ext.C()
        K, Cin, R, S = weight.shape
        w = flat.shadow_storage(weight)  # [Kp][R][S][Cp]
        kp, cp = w.shape[0], w.shape[3]
        xb = as_nhwc(x, cp)
        N, H, W, _ = xb.shape
        P, Q = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
        y = torch.empty(N, P, Q, kp, dtype=torch.bfloat16, device=x.device)
        b = flat.master_storage(bias) if bias is not None else None
        epi = (C.EPI_BIAS_RELU if relu else C.EPI_BIAS) if b is not None else C.EPI_NONE
        if relu and b is None:
            b = torch.zeros(kp, dtype=torch.float32, device=x.device)
            epi = C.EPI_BIAS_RELU
        xs, packed = None, False
        if (epi == C.EPI_NONE and cp == 8 and R == 7 and S == 7 and stride == 2
                and C.stem_s2d_fwd_ok(N, H, W, cp, kp, R, S, stride, pad, Cin)):
            # a 7x7 / 2 stem: the forward runs on the packed space-to-depth image, which the weight
            # gradient then reuses (conv_stem.hip conv_s2d_ws_kernel / stem_s2d_wgrad_kernel) -- the
            # one a graph's input staging wrote along with x (graphed.static_input), or packed here
            img, ver = getattr(x, "_ldnn_s2d", (None, None))
            if (img is not None and ver == x._version and tuple(img.shape) == (N, P + 3, Q + 3, 16)
                    and img.device == x.device):
                xs, packed = img, True
            else:
                xs = torch.empty(N, P + 3, Q + 3, 16, dtype=torch.bfloat16, device=x.device)
        if _fused_bn_ok(bn, K, kp, bias, relu):
            # the conv epilogue accumulates + finalizes the next BN's batch statistics
            args, state = _conv_bn_stats(bn, K, x.device, C)
            done = C.conv_fwd(xb, w, y, stride, pad, b, epi, real_channels=Cin, s2d_xs=xs, s2d_packed=packed,
                              **{"bn_" + k: v for k, v in args.items()})
            _conv_bn_stats_done(bn, done, y, state)
        else:
            C.conv_fwd(xb, w, y, stride, pad, b, epi, real_channels=Cin, s2d_xs=xs, s2d_packed=packed)
        ctx.save_for_backward(xb, y, xs)
        ctx.meta = (stride, pad, flat, weight, bias, relu, Cin, x.dtype)
        src = getattr(x, "_ldnn_bnsrc", None)
        ctx.bnsrc = src if (CONV_BN_BWD and src is not None and stride == 1 and src.C == cp == Cin) else None
        return nchw_view(y, K)

    @staticmethod
    def backward(ctx, gy):
        C = _ext.C()
        xb, y, xs = ctx.saved_tensors
        stride, pad, flat, weight, bias, relu, Cin, in_dtype = ctx.meta
        kp = y.shape[3]
        g = as_nhwc(gy if gy.dtype == torch.bfloat16 else gy.to(torch.bfloat16), kp)
        if relu:
            gz = torch.empty_like(y)
            if bias is not None:   # ReLU backward + the bias gradient's column sums in one pass
                C.act_bwd_colsum(g.contiguous().view(-1, kp), y.view(-1, kp), gz.view(-1, kp),
                                 flat.grad_storage(bias), 0, flat.grad_beta(bias) != 0.0,
                                 ws=_colsum_ws(flat, bias, kp, y.device))
            else:
                C.act_bwd(g.contiguous(), y, gz, 0)
            g = gz
        elif bias is not None:
            C.colsum(g.contiguous().view(-1, kp), flat.grad_storage(bias), flat.grad_beta(bias) != 0.0,
                     ws=_colsum_ws(flat, bias, kp, g.device))
        dw, beta = flat.grad_storage(weight), flat.grad_beta(weight)
        dx = None
        if ctx.needs_input_grad[0]:
            # dgrad + wgrad of the layer: one launch where the kernels allow (conv_bwd)
            dxb = torch.empty_like(xb)
            src = ctx.bnsrc
            kw = src.dgrad_kwargs() if src is not None and not src.twin_used else None
            if C.conv_bwd(g, flat.shadow_storage(weight), dxb, xb, dw, stride, pad, beta, Cin, **(kw or {})) and kw:
                # the BN's backward finds its statistics finalized if this dx reaches it unchanged
                src.pre = (dxb.data_ptr(), dxb._version)
            ctx.bnsrc = None
            dx = _zpad(nchw_view(dxb, Cin))   # (weight pad channels are zero)
            if in_dtype != torch.bfloat16:
                dx = dx.to(in_dtype)
        else:
            C.conv_wgrad(g, xb, dw, stride, pad, beta, real_channels=Cin, s2d_xs=xs)
        flat.notify(weight, bias)
        return dx, None, None, None, None, None, None, None


class _Conv2dPairNative(torch.autograd.Function):
    """A downsampling residual block's two convolutions of one input -- the 3x3 (conv0 on x) and
    the 1x1 shortcut (conv1 on x's twin xt) -- as ONE forward launch (conv_fwd2: both GEMMs share
    the chip), each with its BN's fused statistics; the backward runs each conv's dgrad + wgrad
    pair and returns the two input gradients separately (the producer sums them)."""

    @staticmethod
    def forward(ctx, x, xt, w0, w1, flat, meta0, meta1):
        C = _ext.C()
        (st0, p0, bn0), (st1, p1, bn1) = meta0, meta1
        sh0, sh1 = flat.shadow_storage(w0), flat.shadow_storage(w1)
        (kp0, cp), kp1 = (sh0.shape[0], sh0.shape[3]), sh1.shape[0]
        K0, Cin, R0, S0 = w0.shape
        K1, _, R1, S1 = w1.shape
        xb = as_nhwc(x, cp)
        N, H, W, _ = xb.shape
        dev = x.device
        ys, args, states = [], [], []
        for (K, kp, R, S, st, pd, bn) in ((K0, kp0, R0, S0, st0, p0, bn0), (K1, kp1, R1, S1, st1, p1, bn1)):
            P, Q = (H + 2 * pd - R) // st + 1, (W + 2 * pd - S) // st + 1
            ys.append(torch.empty(N, P, Q, kp, dtype=torch.bfloat16, device=dev))
            a, stt = _conv_bn_stats(bn, K, dev, C) if _fused_bn_ok(bn, K, kp, None, False) else (None, None)
            args.append(a)
            states.append(stt)
        done = C.conv_fwd2(xb, sh0, ys[0], st0, p0, sh1, ys[1], st1, p1, args[0], args[1])
        for bn, d, y, stt in zip((bn0, bn1), done, ys, states):
            if stt is not None:
                _conv_bn_stats_done(bn, d, y, stt)
        ctx.save_for_backward(xb)
        ctx.meta = (flat, (w0, st0, p0), (w1, st1, p1), Cin, x.dtype)
        return nchw_view(ys[0], K0), nchw_view(ys[1], K1)

    @staticmethod
    def backward(ctx, g0, g1):
        C = _ext.C()
        (xb,) = ctx.saved_tensors
        flat, c0, c1, Cin, in_dtype = ctx.meta
        if g0 is not None and g1 is not None and ctx.needs_input_grad[0] and ctx.needs_input_grad[1]:
            # both convs' dgrads and wgrads in one launch (conv_bwd2)
            job = []
            for g, (weight, st, pd) in ((g0, c0), (g1, c1)):
                sh = flat.shadow_storage(weight)
                gb = as_nhwc(g if g.dtype == torch.bfloat16 else g.to(torch.bfloat16), sh.shape[0])
                job.append((gb, sh, torch.empty_like(xb), flat.grad_storage(weight), st, pd, flat.grad_beta(weight)))
            (ga, sa, xa, wa, sta, pa, ba), (gc, sc, xc, wc, stc, pc, bc) = job
            C.conv_bwd2(xb, ga, sa, xa, wa, sta, pa, ba, gc, sc, xc, wc, stc, pc, bc, Cin)
            flat.notify(c0[0], c1[0])
            dxs = [_zpad(nchw_view(xa, Cin)), _zpad(nchw_view(xc, Cin))]
            if in_dtype != torch.bfloat16:
                dxs = [d.to(in_dtype) for d in dxs]
            return dxs[0], dxs[1], None, None, None, None, None
        dxs = []
        for k, (g, (weight, st, pd)) in enumerate(((g0, c0), (g1, c1))):
            if g is None:
                dxs.append(None)
                continue
            sh = flat.shadow_storage(weight)
            gb = as_nhwc(g if g.dtype == torch.bfloat16 else g.to(torch.bfloat16), sh.shape[0])
            dw, beta = flat.grad_storage(weight), flat.grad_beta(weight)
            if ctx.needs_input_grad[k]:
                dxb = torch.empty_like(xb)
                C.conv_bwd(gb, sh, dxb, xb, dw, st, pd, beta, Cin)
                dx = _zpad(nchw_view(dxb, Cin))
                dxs.append(dx if in_dtype == torch.bfloat16 else dx.to(in_dtype))
            else:
                C.conv_wgrad(gb, xb, dw, st, pd, beta, real_channels=Cin)
                dxs.append(None)
            flat.notify(weight)
        return dxs[0], dxs[1], None, None, None, None, None


def conv2d_pair(x, xt, mod0, mod1):
    """(mod0(x), mod1(xt)) -- a downsampling block's 3x3 conv and 1x1 shortcut conv of one input
    (xt: x's twin, LF.shortcut_input) -- as one native forward launch on the GPU (both bias-free,
    no fused ReLU); otherwise the two module calls."""
    if _ext.use_native(x) and xt.data_ptr() == x.data_ptr():
        flat = getattr(mod0, "_ldnn_flat", None)
        ok = (flat is not None and flat.shadow is not None and getattr(mod1, "_ldnn_flat", None) is flat
              and all(m.groups == 1 and m.dilation == (1, 1) and m.bias is None and m.stride[0] == m.stride[1]
                      and isinstance(m.padding, tuple) and m.padding[0] == m.padding[1]
                      and getattr(m, "activation", None) != "relu" for m in (mod0, mod1))
              and mod0.in_channels == mod1.in_channels)
        if ok and _fire_pre_hooks((mod0, mod1), x):
            bn0 = mod0._ldnn_stats_bn if _layers_fuse_bn_stats() else None
            bn1 = mod1._ldnn_stats_bn if _layers_fuse_bn_stats() else None
            y0, y1 = _Conv2dPairNative.apply(x, xt, mod0.weight, mod1.weight, flat,
                                             (mod0.stride[0], mod0.padding[0], bn0),
                                             (mod1.stride[0], mod1.padding[0], bn1))
            return _zpad(y0), _zpad(y1)
    return mod0(x), mod1(xt)


def _layers_fuse_bn_stats() -> bool:
    from ..models import layers
    return layers.FUSE_BN_STATS


def conv2d(x, mod, relu: bool = False, bn=None):
    """Convolution of module `mod` (nn.Conv2d parameters).  GPU: native implicit-GEMM
    kernels on NHWC bf16 activations and KRSC bf16 weights (groups=1, dilation=1);
    CPU: the fp32 reference."""
    if _ext.use_native(x):
        flat = getattr(mod, "_ldnn_flat", None)
        ok = (flat is not None and flat.shadow is not None and mod.groups == 1 and mod.dilation == (1, 1)
              and mod.stride[0] == mod.stride[1] and mod.padding[0] == mod.padding[1]
              and isinstance(mod.padding, tuple))
        if not ok:
            raise RuntimeError("native conv needs groups=1, dilation=1, square stride/padding and "
                               "the model attached to FlatParams (ldnn.prepare(model))")
        # output pad channels: zero weight rows and bias entries -> exactly 0 (also after ReLU)
        return _zpad(_Conv2dNative.apply(x, mod.weight, mod.bias, mod.stride[0], mod.padding[0], flat, relu, bn))
    y = F.conv2d(x.float(), mod.weight, mod.bias, mod.stride, mod.padding, mod.dilation, mod.groups)
    return F.relu(y) if relu else y


def _bn_workspace(mod, C: int, dev, C_) -> torch.Tensor:
    """The module's persistent BN workspace (zeroed once: the kernels keep their
    accumulators clear), so a BN costs no zero-fill launch per call."""
    ws = getattr(mod, "_ldnn_bn_ws", None)
    n = C_.bn_workspace_floats(C)
    if ws is None or ws.device != dev or ws.numel() < n:
        ws = torch.zeros(n, dtype=torch.float32, device=dev)
        mod._ldnn_bn_ws = ws
    return ws


def _with_twin(y: torch.Tensor, twin: torch.Tensor) -> torch.Tensor:
    """Native BN / pool outputs come with a twin: a second autograd output over the
    same storage.  A residual block reads its shortcut through the twin
    (``shortcut_input``), so the producer's backward receives the two branch
    gradients separately and sums them inside its own kernels -- no separate
    elementwise add of the gradients (autograd's accumulation of a tensor used twice)."""
    y._ldnn_twin = twin
    return y


def shortcut_input(x: torch.Tensor) -> torch.Tensor:
    """The tensor a residual block's shortcut branch should read (x's twin if it has one)."""
    t = getattr(x, "_ldnn_twin", None)
    src = getattr(x, "_ldnn_bnsrc", None)
    if src is not None:   # the producer BN's gradient arrives in two parts: no dgrad-side statistics
        src.twin_used = True
    return x if t is None else t


class _BatchNormNative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, mod, flat, relu):
        C_ = _ext.C()
        N, C, H, W = x.shape
        xb = as_nhwc(x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16), C, zero_pad=False)
        x2 = xb.view(-1, C)
        r2 = None
        if residual is not None:
            rb = residual if residual.dtype == torch.bfloat16 else residual.to(torch.bfloat16)
            r2 = as_nhwc(rb, C, zero_pad=False).reshape(-1, C)
        y = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=x.device)
        dev = x.device
        ws = _bn_workspace(mod, C, dev, C_)
        smean = torch.empty(C, dtype=torch.float32, device=dev)
        sinv = torch.empty(C, dtype=torch.float32, device=dev)
        gamma = flat.master_storage(weight)[:C] if weight is not None else None
        beta = flat.master_storage(bias)[:C] if bias is not None else None
        training = mod.training or not mod.track_running_stats
        # ReLU as a bit mask for the backward (its reduce and apply passes read 1/16 of
        # y's bytes); only when a backward will run
        mask = (torch.empty(x2.shape[0] * C // 8, dtype=torch.uint8, device=dev)
                if relu and any(ctx.needs_input_grad) and BN_RELU_MASK else None)
        pre = mod.__dict__.pop("_ldnn_pre", None)
        if pre is not None and mod.training and pre[0] == x2.data_ptr():
            # statistics already accumulated + finalized by the producing conv's epilogue
            smean, sinv = pre[1], pre[2]
            C_.bn_fwd(x2, y.view(-1, C), r2, gamma, beta, None, None, smean, sinv, ws, mod.eps, 0.0, True, relu,
                      None, stats_ready=True, mask=mask)
        else:
            rm, rv, mom, nbt = _bn_train_state(mod, dev)
            C_.bn_fwd(x2, y.view(-1, C), r2, gamma, beta, rm if (training and mod.training) or not training else None,
                      rv if (training and mod.training) or not training else None, smean, sinv, ws, mod.eps,
                      mom or 0.0, training, relu, nbt, mask=mask)
        ctx.mask = mask
        ctx.save_for_backward(x2, y if mask is None else x2.new_empty(0), smean, sinv)
        ctx.meta = (flat, weight, bias, relu, residual is not None, ws, (N, C, H, W), x.dtype)
        ctx.set_materialize_grads(False)
        out = nchw_view(y, C)
        ctx.bnsrc = None
        if (CONV_BN_BWD and mod.training and weight is not None and bias is not None
                and (mask is not None or not relu) and any(ctx.needs_input_grad)):
            ctx.bnsrc = out._ldnn_bnsrc = _BnBwdSrc(mod, flat, weight, bias, x2, mask, smean, sinv, ws, C)
        return out, nchw_view(y, C)

    @staticmethod
    def backward(ctx, gy, gy_twin):
        C_ = _ext.C()
        x2, y, smean, sinv = ctx.saved_tensors
        flat, weight, bias, relu, has_res, ws, (N, C, H, W), in_dtype = ctx.meta
        if gy is None:
            gy, gy_twin = gy_twin, None
        if gy is None:
            return None, None, None, None, None, None, None
        g2 = as_nhwc(gy if gy.dtype == torch.bfloat16 else gy.to(torch.bfloat16), C, zero_pad=False)
        g2 = g2.contiguous().view(-1, C)
        gt = None
        if gy_twin is not None:   # the shortcut branch's gradient of the same output: summed in the kernels
            gt = as_nhwc(gy_twin if gy_twin.dtype == torch.bfloat16 else gy_twin.to(torch.bfloat16), C,
                         zero_pad=False).contiguous().view(-1, C)
        dx = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=x2.device)
        dres = torch.empty_like(dx) if has_res and ctx.needs_input_grad[3] else None
        gamma = flat.master_storage(weight)[:C] if weight is not None else None
        dg = flat.grad_storage(weight)[:C] if weight is not None else None
        db = flat.grad_storage(bias)[:C] if bias is not None else None
        # first write of the step: the finalize stores dgamma / dbeta instead of adding
        fresh = [(t, flat.grad_beta(p) == 0.0) for t, p in ((dg, weight), (db, bias)) if p is not None]
        assign = all(f for _, f in fresh)
        if not assign:  # mixed (only if a caller accumulated one of them): clear the fresh ones
            for t, f in fresh:
                if f:
                    t.zero_()
        mask = ctx.mask
        yv = y.view(-1, C) if mask is None else x2   # (y is not read when the mask is given)
        pre = ctx.bnsrc.pre if ctx.bnsrc is not None else None
        ctx.bnsrc = None
        # statistics finalized by the consumer conv's dgrad epilogue, if its dx arrived unchanged
        # (a second consumer's gradient -- an in-place accumulation bumps the version -- or a
        # twin branch gradient sends the BN through its own reduce)
        ready = (pre is not None and gt is None and assign and pre[0] == g2.data_ptr() and pre[1] == gy._version)
        BN_BWD_FUSED[0] += int(ready)
        C_.bn_bwd(x2, yv, g2, dx.view(-1, C), dres.view(-1, C) if dres is not None else None, gamma,
                  smean, sinv, ws, dg, db, relu, mask=mask, grad_assign=assign, dy2=gt, stats_ready=ready)
        flat.notify(weight, bias)
        dxv = nchw_view(dx, C)
        dresv = nchw_view(dres, C) if dres is not None else None
        if in_dtype != torch.bfloat16:
            dxv = dxv.to(in_dtype)
        return dxv, None, None, dresv, None, None, None


class _BatchNormDualNative(torch.autograd.Function):
    """relu(bn_a(x) + bn_b(r)) -- a residual block whose shortcut carries its own BatchNorm
    (1x1 downsample conv + BN) -- as one native pass each way (bn_pool.hip bn_dual_*): the
    shortcut BN's output is never stored, both BNs' backward statistics come from one
    reduce pass over the shared post-ReLU gradient, and one apply pass writes dx and dr."""

    @staticmethod
    def forward(ctx, x, r, wa, ba, wb, bb, mod_a, mod_b, flat):
        C_ = _ext.C()
        N, C, H, W = x.shape
        dev = x.device
        x2 = as_nhwc(x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16), C, zero_pad=False).reshape(-1, C)
        r2 = as_nhwc(r if r.dtype == torch.bfloat16 else r.to(torch.bfloat16), C, zero_pad=False).reshape(-1, C)
        y = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=dev)
        mask = (torch.empty(x2.shape[0] * C // 8, dtype=torch.uint8, device=dev)
                if any(ctx.needs_input_grad) and BN_RELU_MASK else None)

        def state(mod, t2, w, b):
            st = dict(ws=_bn_workspace(mod, C, dev, C_), gamma=flat.master_storage(w)[:C],
                      beta=flat.master_storage(b)[:C])
            pre = mod.__dict__.pop("_ldnn_pre", None)
            if pre is not None and pre[0] == t2.data_ptr():
                # statistics already accumulated + finalized by the producing conv's epilogue
                st.update(rm=None, rv=None, mom=0.0, nb=None, mean=pre[1], invstd=pre[2], ready=True)
            else:
                rm, rv, mom, nbt = _bn_train_state(mod, dev)
                st.update(rm=rm, rv=rv, mom=mom or 0.0, nb=nbt, mean=torch.empty(C, dtype=torch.float32, device=dev),
                          invstd=torch.empty(C, dtype=torch.float32, device=dev), ready=False)
            return st

        sa, sb = state(mod_a, x2, wa, ba), state(mod_b, r2, wb, bb)
        C_.bn_dual_fwd(x2, r2, y.view(-1, C), mask,
                       sa["gamma"], sa["beta"], sa["rm"], sa["rv"], sa["mean"], sa["invstd"], sa["ws"], mod_a.eps,
                       sa["mom"], sa["nb"], sa["ready"],
                       sb["gamma"], sb["beta"], sb["rm"], sb["rv"], sb["mean"], sb["invstd"], sb["ws"], mod_b.eps,
                       sb["mom"], sb["nb"], sb["ready"])
        ctx.mask = mask
        ctx.save_for_backward(x2, r2, y.view(-1, C) if mask is None else x2.new_empty(0), sa["mean"], sa["invstd"],
                              sb["mean"], sb["invstd"])
        ctx.meta = (flat, (wa, ba, sa["ws"]), (wb, bb, sb["ws"]), (N, C, H, W), x.dtype, r.dtype)
        ctx.set_materialize_grads(False)
        return nchw_view(y, C), nchw_view(y, C)

    @staticmethod
    def backward(ctx, gy, gy_twin):
        C_ = _ext.C()
        x2, r2, y2, mean_a, inv_a, mean_b, inv_b = ctx.saved_tensors
        flat, (wa, ba, ws_a), (wb, bb, ws_b), (N, C, H, W), x_dtype, r_dtype = ctx.meta
        if gy is None:
            gy, gy_twin = gy_twin, None
        if gy is None:
            return (None,) * 9

        def nhwc2(t):
            return as_nhwc(t if t.dtype == torch.bfloat16 else t.to(torch.bfloat16), C,
                           zero_pad=False).contiguous().view(-1, C)

        g2 = nhwc2(gy)
        gt = nhwc2(gy_twin) if gy_twin is not None else None
        dx = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=x2.device)
        dr = torch.empty_like(dx)

        def grads(w, b):
            dg, db = flat.grad_storage(w)[:C], flat.grad_storage(b)[:C]
            fresh = [(dg, flat.grad_beta(w) == 0.0), (db, flat.grad_beta(b) == 0.0)]
            assign = all(f for _, f in fresh)
            if not assign:   # mixed (only if a caller accumulated one of them): clear the fresh ones
                for t, f in fresh:
                    if f:
                        t.zero_()
            return flat.master_storage(w)[:C], dg, db, assign

        ga, dga, dba, asa = grads(wa, ba)
        gb, dgb, dbb, asb = grads(wb, bb)
        C_.bn_dual_bwd(x2, r2, y2 if ctx.mask is None else x2, ctx.mask, g2, gt, dx.view(-1, C), dr.view(-1, C),
                       ga, mean_a, inv_a, ws_a, dga, dba, asa, gb, mean_b, inv_b, ws_b, dgb, dbb, asb)
        flat.notify(wa, ba)
        flat.notify(wb, bb)
        dxv, drv = nchw_view(dx, C), nchw_view(dr, C)
        if x_dtype != torch.bfloat16:
            dxv = dxv.to(x_dtype)
        if r_dtype != torch.bfloat16:
            drv = drv.to(r_dtype)
        return dxv, drv, None, None, None, None, None, None, None


# y = relu(bn_a(x) + bn_b(r)) in one pass (LDNN_BN_DUAL=0: bn_b's apply + bn_a's residual pass)
BN_DUAL_FUSED = __import__("os").environ.get("LDNN_BN_DUAL", "1") != "0"


def batch_norm_dual_act(x, mod_a, r, mod_b):
    """relu(mod_a(x) + mod_b(r)): the tail of a residual block whose shortcut is conv + BN."""
    fa, fb = getattr(mod_a, "_ldnn_flat", None), getattr(mod_b, "_ldnn_flat", None)
    ok = (BN_DUAL_FUSED and _ext.use_native(x) and fa is not None and fa is fb and mod_a.training
          and mod_b.training and mod_a.affine and mod_b.affine and x.dim() == 4 and x.shape == r.shape
          and x.shape[1] % 8 == 0)
    if ok:
        return _with_twin(*_BatchNormDualNative.apply(x, r, mod_a.weight, mod_a.bias, mod_b.weight, mod_b.bias,
                                                      mod_a, mod_b, fa))
    return mod_a.act(x, residual=mod_b(r), relu=True)


# BatchNorm + ReLU keeps a bit mask of the output for its backward (measured A/B in
# profiles/, LDNN_BN_RELU_MASK=0 reads the bf16 output instead)
BN_RELU_MASK = __import__("os").environ.get("LDNN_BN_RELU_MASK", "1") != "0"


def batch_norm_act(x, mod, residual=None, relu: bool = False):
    """relu?(BatchNorm2d(x) (+ residual)) -- fused into one native pass on the GPU
    (fp32 statistics over NHWC bf16); the CPU path is the fp32 reference."""
    flat = getattr(mod, "_ldnn_flat", None)
    if _ext.use_native(x) and flat is not None and x.shape[1] % 8 == 0 and mod.affine:
        return _with_twin(*_BatchNormNative.apply(x, mod.weight, mod.bias, residual, mod, flat, relu))
    y = batch_norm2d(x, mod)
    if residual is not None:
        y = y + residual
    return F.relu(y) if relu else y


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


# ------------------------------------------------------------------ pooling
class _PoolNative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, stride, pad, is_max):
        C_ = _ext.C()
        N, C, H, W = x.shape
        cp = _up8(C)
        xb = as_nhwc(x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16), cp)
        P, Q = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
        y = torch.empty(N, P, Q, cp, dtype=torch.bfloat16, device=x.device)
        am = torch.empty(N, P, Q, cp, dtype=torch.uint8, device=x.device) if is_max else None
        C_.pool_fwd(xb.contiguous(), y, am, k, k, stride, pad, is_max)
        ctx.save_for_backward(am) if is_max else None
        ctx.meta = (k, stride, pad, is_max, (N, C, H, W, cp), x.dtype)
        ctx.set_materialize_grads(False)
        return nchw_view(y, C), nchw_view(y, C)

    @staticmethod
    def backward(ctx, gy, gy_twin):
        C_ = _ext.C()
        k, stride, pad, is_max, (N, C, H, W, cp), in_dtype = ctx.meta
        if gy is None:
            gy, gy_twin = gy_twin, None
        if gy is None:
            return None, None, None, None, None
        am = ctx.saved_tensors[0] if is_max else None
        g = as_nhwc(gy if gy.dtype == torch.bfloat16 else gy.to(torch.bfloat16), cp).contiguous()
        gt = None
        if gy_twin is not None:
            gt = as_nhwc(gy_twin if gy_twin.dtype == torch.bfloat16 else gy_twin.to(torch.bfloat16), cp).contiguous()
        dx = torch.empty(N, H, W, cp, dtype=torch.bfloat16, device=gy.device)
        C_.pool_bwd(g, am, dx, k, k, stride, pad, is_max, dy2=gt)
        out = _zpad(nchw_view(dx, C))   # (pooled gradient of zero pad channels)
        return (out if in_dtype == torch.bfloat16 else out.to(in_dtype)), None, None, None, None


class _BnReluMaxPoolNative(torch.autograd.Function):
    """maxpool3x3/2(relu(BatchNorm2d(x))) in one native pass each way (bn_pool.hip
    bn_maxpool_*): the BN output is never stored, the pool's argmax doubles as the
    ReLU mask and the backward turns the pooled gradient straight into dx."""

    @staticmethod
    def forward(ctx, x, weight, bias, mod, flat, pad):
        C_ = _ext.C()
        N, C, H, W = x.shape
        xb = as_nhwc(x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16), C, zero_pad=False).contiguous()
        P, Q = (H + 2 * pad - 3) // 2 + 1, (W + 2 * pad - 3) // 2 + 1
        dev = x.device
        y = torch.empty(N, P, Q, C, dtype=torch.bfloat16, device=dev)
        am = torch.empty(N, P, Q, C, dtype=torch.uint8, device=dev)
        # the BN input at every argmax: the backward statistics read it (pooled size) instead of x
        xam = torch.empty(N, P, Q, C, dtype=torch.bfloat16, device=dev) if BN_POOL_MODE == 1 else None
        ws = _bn_workspace(mod, C, dev, C_)
        gamma = flat.master_storage(weight)[:C] if weight is not None else None
        beta = flat.master_storage(bias)[:C] if bias is not None else None
        pre = mod.__dict__.pop("_ldnn_pre", None)
        if pre is not None and pre[0] == xb.data_ptr():
            # statistics already accumulated + finalized by the producing conv's epilogue
            smean, sinv = pre[1], pre[2]
            C_.bn_pool_fwd(xb, y, am, gamma, beta, None, None, smean, sinv, ws, mod.eps, 0.0, None, True, pad, xam)
        else:
            smean = torch.empty(C, dtype=torch.float32, device=dev)
            sinv = torch.empty(C, dtype=torch.float32, device=dev)
            rm, rv, mom, nbt = _bn_train_state(mod, dev)
            C_.bn_pool_fwd(xb, y, am, gamma, beta, rm, rv, smean, sinv, ws, mod.eps, mom or 0.0, nbt, False, pad, xam)
        ctx.save_for_backward(xb, am, smean, sinv, xam)
        ctx.meta = (flat, weight, bias, ws, pad, C, x.dtype)
        ctx.set_materialize_grads(False)
        return nchw_view(y, C), nchw_view(y, C)

    @staticmethod
    def backward(ctx, gy, gy_twin):
        C_ = _ext.C()
        xb, am, smean, sinv, xam = ctx.saved_tensors
        flat, weight, bias, ws, pad, C, in_dtype = ctx.meta
        if gy is None:
            gy, gy_twin = gy_twin, None
        if gy is None:
            return None, None, None, None, None, None
        g = as_nhwc(gy if gy.dtype == torch.bfloat16 else gy.to(torch.bfloat16), C, zero_pad=False).contiguous()
        gt = None
        if gy_twin is not None:
            gt = as_nhwc(gy_twin if gy_twin.dtype == torch.bfloat16 else gy_twin.to(torch.bfloat16), C,
                         zero_pad=False).contiguous()
        dx = torch.empty_like(xb)
        gamma = flat.master_storage(weight)[:C] if weight is not None else None
        dg = flat.grad_storage(weight)[:C] if weight is not None else None
        db = flat.grad_storage(bias)[:C] if bias is not None else None
        fresh = [(t, flat.grad_beta(p) == 0.0) for t, p in ((dg, weight), (db, bias)) if p is not None]
        assign = all(f for _, f in fresh)
        if not assign:
            for t, f in fresh:
                if f:
                    t.zero_()
        C_.bn_pool_bwd(xb, g, am, dx, gamma, smean, sinv, ws, dg, db, assign, gt, pad, xam)
        flat.notify(weight, bias)
        dxv = nchw_view(dx, C)
        return (dxv if in_dtype == torch.bfloat16 else dxv.to(in_dtype)), None, None, None, None, None


# BN + ReLU + max-pool fused (LDNN_BN_POOL=0: the separate BN-apply and pool passes; 1: fused, the
# backward statistics from the pooled side (x at the argmax); 2: fused, the statistics pass reads x)
BN_POOL_MODE = int(__import__("os").environ.get("LDNN_BN_POOL", "1"))
BN_POOL_FUSED = BN_POOL_MODE != 0


def bn_relu_maxpool(x, bn, pool):
    """pool(relu(bn(x))) for a 3x3 / stride-2 max-pool: one native pass each way on the
    GPU in training mode (C / 8 dividing 256), else the separate layers."""
    flat = getattr(bn, "_ldnn_flat", None)
    k, st, pad = _sq(pool.kernel_size), _sq(pool.stride if pool.stride is not None else pool.kernel_size), \
        _sq(pool.padding)
    C = x.shape[1] if x.dim() == 4 else 0
    ok = (BN_POOL_FUSED and _ext.use_native(x) and flat is not None and bn.training and bn.affine
          and x.dim() == 4 and C % 8 == 0 and 256 % (C // 8 or 1) == 0 and C // 8 <= 256
          and k == 3 and st == 2 and pad is not None and 0 <= pad <= 1 and _sq(pool.dilation) == 1
          and not getattr(pool, "ceil_mode", False) and not getattr(pool, "return_indices", False))
    if ok:
        return _with_twin(*_BnReluMaxPoolNative.apply(x, bn.weight, bn.bias, bn, flat, pad))
    return pool(bn.act(x, relu=True))


def _sq(v):
    return v if isinstance(v, int) else (v[0] if v[0] == v[1] else None)


class _PoolFlatNative(torch.autograd.Function):
    """A pool whose only consumer flattens it (LeNet-5's last pool -> fc1): the kernel
    writes the dense NCHW output itself, so ``flatten(1)`` is a free view instead of an
    NHWC -> NCHW copy, and the backward reads the flattened gradient in place
    (bn_pool.hip pool_fwd_kernel / pool_bwd_kernel with ``cl`` > 0)."""

    @staticmethod
    def forward(ctx, x, k, stride, pad, is_max):
        C_ = _ext.C()
        N, C, H, W = x.shape
        cp = _up8(C)
        xb = as_nhwc(x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16), cp)
        P, Q = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
        y = torch.empty(N, C, P, Q, dtype=torch.bfloat16, device=x.device)
        am = torch.empty(N, P, Q, cp, dtype=torch.uint8, device=x.device) if is_max else None
        C_.pool_fwd(xb.contiguous(), y, am, k, k, stride, pad, is_max, nchw_out=True)
        ctx.save_for_backward(am) if is_max else None
        ctx.meta = (k, stride, pad, is_max, (N, C, H, W, cp), x.dtype)
        return y

    @staticmethod
    def backward(ctx, gy):
        C_ = _ext.C()
        k, stride, pad, is_max, (N, C, H, W, cp), in_dtype = ctx.meta
        am = ctx.saved_tensors[0] if is_max else None
        g = (gy if gy.dtype == torch.bfloat16 else gy.to(torch.bfloat16)).contiguous()
        dx = torch.empty(N, H, W, cp, dtype=torch.bfloat16, device=gy.device)
        C_.pool_bwd(g, am, dx, k, k, stride, pad, is_max, nchw_dy=True)
        out = _zpad(nchw_view(dx, C))
        return (out if in_dtype == torch.bfloat16 else out.to(in_dtype)), None, None, None, None


def pool2d(x, mod, is_max: bool):
    """Max / average pooling.  ``mod.flatten_out`` (set by a model whose pool feeds a
    flatten, e.g. LeNet-5) makes the native path return a dense NCHW tensor."""
    k, st, pad = _sq(mod.kernel_size), _sq(mod.stride if mod.stride is not None else mod.kernel_size), _sq(mod.padding)
    simple = (None not in (k, st, pad) and not getattr(mod, "ceil_mode", False)
              and (not is_max or _sq(mod.dilation) == 1) and (is_max or getattr(mod, "count_include_pad", True))
              and k * k <= 255)
    if _ext.use_native(x) and simple and x.dim() == 4 and getattr(mod, "flatten_out", False):
        return _PoolFlatNative.apply(x, k, st, pad, is_max)
    if _ext.use_native(x) and simple and x.dim() == 4:
        y, twin = _PoolNative.apply(x, k, st, pad, is_max)   # (the input's pad was zeroed / zero)
        return _with_twin(_zpad(y), _zpad(twin))
    if is_max:
        return F.max_pool2d(x, mod.kernel_size, mod.stride, mod.padding, mod.dilation, mod.ceil_mode)
    return F.avg_pool2d(x, mod.kernel_size, mod.stride, mod.padding, mod.ceil_mode, mod.count_include_pad)


class _GapNative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        C_ = _ext.C()
        N, C, H, W = x.shape
        cp = _up8(C)
        xb = as_nhwc(x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16), cp).contiguous()
        y = torch.empty(N, cp, dtype=torch.bfloat16, device=x.device)
        C_.gap_fwd(xb.view(N, H * W, cp), y)
        ctx.meta = (N, C, H, W, cp, x.dtype)
        return y[:, :C].view(N, C, 1, 1)

    @staticmethod
    def backward(ctx, gy):
        C_ = _ext.C()
        N, C, H, W, cp, in_dtype = ctx.meta
        g2 = gy.reshape(N, C)
        if cp == C and g2.dtype == torch.bfloat16 and g2.is_contiguous():
            g = g2   # (the Linear dgrad's dense output: no zero-pad copy)
        else:
            g = torch.zeros(N, cp, dtype=torch.bfloat16, device=gy.device)
            g[:, :C] = g2
        dx = torch.empty(N, H, W, cp, dtype=torch.bfloat16, device=gy.device)
        C_.gap_bwd(g, dx.view(N, H * W, cp))
        out = nchw_view(dx, C)
        return out if in_dtype == torch.bfloat16 else out.to(in_dtype)


def adaptive_avg_pool2d(x, output_size):
    os_ = output_size if isinstance(output_size, int) else (output_size[0] if output_size[0] == output_size[1] else None)
    if _ext.use_native(x) and os_ == 1 and x.dim() == 4:
        return _GapNative.apply(x)
    return F.adaptive_avg_pool2d(x, output_size)


class _GapLinearNative(torch.autograd.Function):
    """AdaptiveAvgPool2d(1) -> flatten -> Linear (<= 16 classes) in one launch each way
    (gap_head.hip): the CNN classifier heads at small batch are pure launch latency."""

    @staticmethod
    def forward(ctx, x, weight, bias, flat):
        C_ = _ext.C()
        N, C, H, W = x.shape
        w = flat.shadow_storage(weight)
        npad = w.shape[0]
        xb = as_nhwc(x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16), C).contiguous()
        pooled = torch.empty(N, C, dtype=torch.bfloat16, device=x.device)
        logits = torch.empty(N, npad, dtype=torch.bfloat16, device=x.device)
        b = flat.master_storage(bias) if bias is not None else None
        ncls = weight.shape[0]
        C_.gap_linear_fwd(xb.view(N, H * W, C), w, b, pooled, logits, ncls)
        ctx.save_for_backward(pooled)
        ctx.meta = (N, C, H, W, ncls, x.dtype)
        ctx.flat, ctx.weight, ctx.bias = flat, weight, bias
        return logits[:, :ncls]

    @staticmethod
    def backward(ctx, gy):
        C_ = _ext.C()
        (pooled,) = ctx.saved_tensors
        N, C, H, W, ncls, in_dtype = ctx.meta
        flat, weight, bias = ctx.flat, ctx.weight, ctx.bias
        g = gy if (gy.dtype == torch.bfloat16 and gy.stride(1) == 1) else gy.to(torch.bfloat16).contiguous()
        dx = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=gy.device)
        C_.gap_linear_bwd(g, pooled, flat.shadow_storage(weight), flat.grad_storage(weight),
                          flat.grad_storage(bias) if bias is not None else None, dx.view(N, H * W, C), ncls,
                          beta_w=flat.grad_beta(weight), beta_b=flat.grad_beta(bias) if bias is not None else 0.0)
        flat.notify(weight, bias)
        out = nchw_view(dx, C)
        return (out if in_dtype == torch.bfloat16 else out.to(in_dtype)), None, None, None


# LDNN_GAP_LINEAR=0: the pooled classifier head runs as separate pool + Linear ops (A/B knob)
GAP_LINEAR = os.environ.get("LDNN_GAP_LINEAR", "1") == "1"


def gap_linear(x, pool, fc):
    """fc(flatten(pool(x))) for a global average pool `pool` and an ldnn Linear `fc`; one fused
    launch each way when the shapes allow (<= 16 classes, unpadded features), else the two ops."""
    flat = getattr(fc, "_ldnn_flat", None)
    os_ = pool.output_size if isinstance(pool.output_size, int) else (
        pool.output_size[0] if pool.output_size[0] == pool.output_size[1] else None)
    if (GAP_LINEAR and _ext.use_native(x) and x.dim() == 4 and os_ == 1 and flat is not None
            and flat.shadow is not None and getattr(fc, "activation", "none") == "none"):
        N, C, H, W = x.shape
        w = flat.shadow_storage(fc.weight)
        if (w.shape[1] == C and C == fc.in_features and _ext.C().gap_linear_ok(N, H * W, C, fc.out_features)
                and _fire_pre_hooks((pool, fc), x)):
            return _GapLinearNative.apply(x, fc.weight, fc.bias, flat)
    y = pool(x)
    return fc(y.reshape(y.size(0), -1))
