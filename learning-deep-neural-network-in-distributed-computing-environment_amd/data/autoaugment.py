"""AutoAugment(CIFAR10) for the device-resident loader.

The reference trains on ``transforms.AutoAugment(AutoAugmentPolicy.CIFAR10)`` +
ToTensor + Normalize, run per image by PIL on the CPU inside a num_workers=0
DataLoader (BAR/dataloader.py:14-21; SURVEY Q9: input-bound).  Here the whole
augmentation runs in ONE native kernel (csrc/kernels/augment.hip): a workgroup
per image gathers its uint8 pixels from the resident dataset into LDS, applies
the sampled sub-policy's two ops there (per-channel reductions for Contrast /
AutoContrast / Equalize in LDS), optionally flip+crops, normalises and writes the
bf16/fp32 batch -- no host work per batch.

This module holds the policy (25 sub-policies of two (op, probability,
magnitude-bin) triples), the magnitude tables (10 bins, as torchvision's
``_augmentation_space``), the per-sample counter-based RNG, and a NumPy
implementation of every op with exactly the kernel's arithmetic.  The NumPy code
is the kernel's numerics reference in tests and the CPU fallback.

Op semantics follow torchvision's tensor implementations (nearest-neighbour
affine ops with zero fill, ``_blend`` truncation to uint8, grayscale
0.2989/0.587/0.114, the 3x3 [1 1 1; 1 5 1; 1 1 1]/13 sharpness kernel on the
interior, torchvision's equalize LUT).  torchvision is not importable here, so
bit-parity with it is unpinned; the tests pin kernel == this reference.
"""
from __future__ import annotations

import math

import numpy as np

OPS = ["ShearX", "ShearY", "TranslateX", "TranslateY", "Rotate", "Brightness", "Color", "Contrast", "Sharpness",
       "Posterize", "Solarize", "AutoContrast", "Equalize", "Invert", "Identity"]
OP = {n: i for i, n in enumerate(OPS)}
SIGNED = {"ShearX", "ShearY", "TranslateX", "TranslateY", "Rotate", "Brightness", "Color", "Contrast", "Sharpness"}

# AutoAugmentPolicy.CIFAR10: 25 sub-policies x 2 (op, probability, magnitude bin)
CIFAR10_POLICY = [
    (("Invert", 0.1, None), ("Contrast", 0.2, 6)),
    (("Rotate", 0.7, 2), ("TranslateX", 0.3, 9)),
    (("Sharpness", 0.8, 1), ("Sharpness", 0.9, 3)),
    (("ShearY", 0.5, 8), ("TranslateY", 0.7, 9)),
    (("AutoContrast", 0.5, None), ("Equalize", 0.9, None)),
    (("ShearY", 0.2, 7), ("Posterize", 0.3, 7)),
    (("Color", 0.4, 3), ("Brightness", 0.6, 7)),
    (("Sharpness", 0.3, 9), ("Brightness", 0.7, 9)),
    (("Equalize", 0.6, None), ("Equalize", 0.5, None)),
    (("Contrast", 0.6, 7), ("Sharpness", 0.6, 5)),
    (("Color", 0.7, 7), ("TranslateX", 0.5, 8)),
    (("Equalize", 0.3, None), ("AutoContrast", 0.4, None)),
    (("TranslateY", 0.4, 3), ("Sharpness", 0.2, 6)),
    (("Brightness", 0.9, 6), ("Color", 0.2, 8)),
    (("Solarize", 0.5, 2), ("Invert", 0.0, None)),
    (("Equalize", 0.2, None), ("AutoContrast", 0.6, None)),
    (("Equalize", 0.2, None), ("Equalize", 0.6, None)),
    (("Color", 0.9, 9), ("Equalize", 0.6, None)),
    (("AutoContrast", 0.8, None), ("Solarize", 0.2, 8)),
    (("Brightness", 0.1, 3), ("Color", 0.7, 0)),
    (("Solarize", 0.4, 5), ("AutoContrast", 0.9, None)),
    (("TranslateY", 0.9, 9), ("TranslateY", 0.7, 9)),
    (("AutoContrast", 0.9, None), ("Solarize", 0.8, 3)),
    (("Equalize", 0.8, None), ("Invert", 0.1, None)),
    (("TranslateY", 0.7, 9), ("AutoContrast", 0.9, None)),
]
NUM_BINS = 10
NUM_POLICIES = len(CIFAR10_POLICY)

# modes of the augment kernel
MODE_AUTOAUGMENT = 1
MODE_FLIP_CROP = 2


def _linspace32(a, b, n=NUM_BINS):
    """torch.linspace(a, b, n) in float32 (first half from the start, second half from the end)."""
    step = (b - a) / (n - 1)
    out = np.empty(n, np.float32)
    for i in range(n):
        out[i] = np.float32(a + i * step) if i < n // 2 else np.float32(b - (n - 1 - i) * step)
    return out


def magnitude_table(H: int, W: int) -> np.ndarray:
    """[15 ops][10 bins] float32 magnitudes (torchvision _augmentation_space)."""
    t = np.zeros((len(OPS), NUM_BINS), np.float32)
    t[OP["ShearX"]] = t[OP["ShearY"]] = _linspace32(0.0, 0.3)
    t[OP["TranslateX"]] = _linspace32(0.0, 150.0 / 331.0 * W)
    t[OP["TranslateY"]] = _linspace32(0.0, 150.0 / 331.0 * H)
    t[OP["Rotate"]] = _linspace32(0.0, 30.0)
    for n in ("Brightness", "Color", "Contrast", "Sharpness"):
        t[OP[n]] = _linspace32(0.0, 0.9)
    t[OP["Posterize"]] = 8 - np.round(np.arange(NUM_BINS) / ((NUM_BINS - 1) / 4)).astype(np.float32)
    t[OP["Solarize"]] = _linspace32(255.0, 0.0)
    return t


def policy_table(policy=CIFAR10_POLICY):
    """(op ids [P*2] int32, probabilities [P*2] float32, bins [P*2] int32, signed [15] int32)."""
    ops = np.array([OP[o] for sp in policy for (o, _, _) in sp], np.int32)
    prob = np.array([p for sp in policy for (_, p, _) in sp], np.float32)
    bins = np.array([(-1 if m is None else m) for sp in policy for (_, _, m) in sp], np.int32)
    signed = np.array([1 if n in SIGNED else 0 for n in OPS], np.int32)
    return ops, prob, bins, signed


# ---------------------------------------------------------------- RNG
_M64 = (1 << 64) - 1


def smix(z: int) -> int:
    """splitmix64 finaliser (same as the kernel's)."""
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def draws(seed: int, b: int) -> dict:
    """Per-sample random choices of sample b of a batch with batch seed `seed`."""
    h0 = smix((seed ^ ((b * 0xD1B54A32D192ED03) & _M64)) & _M64)
    h1 = smix(h0)
    return dict(policy=(h0 >> 32) % NUM_POLICIES,
                u=(np.float32((h0 & 0xFFFFFF) * (1.0 / 16777216.0)), np.float32((h1 >> 40) * (1.0 / 16777216.0))),
                sign=((h1 >> 1) & 1, (h1 >> 2) & 1), flip=(h1 >> 3) & 1, dy=(h1 >> 8) & 0xFF, dx=(h1 >> 16) & 0xFF)


def batch_seed(loader_seed: int, epoch: int, batch: int) -> int:
    """63-bit seed of one batch (fits the kernel binding's int64)."""
    return smix(((loader_seed & 0xFFFFFFFF) << 32) ^ ((epoch & 0xFFFF) << 16) ^ (batch & 0xFFFF)) >> 1


# ---------------------------------------------------------------- ops (NumPy, float32 like the kernel)
f32 = np.float32


def _blend_coefs(ratio_f32):
    r = 1.0 + float(ratio_f32)  # torchvision: ratio = 1.0 + magnitude (Python float)
    return f32(r), f32(1.0 - r)


def _blend(img, other, ratio_f32):
    c1, c2 = _blend_coefs(ratio_f32)
    v = c1 * img.astype(f32) + c2 * other.astype(f32)
    return np.clip(v, f32(0), f32(255)).astype(np.uint8)


def _gray(img):
    if img.shape[0] == 1:
        return img[0].copy()
    r, g, b = (img[i].astype(f32) for i in range(3))
    return (f32(0.2989) * r + f32(0.587) * g + f32(0.114) * b).astype(np.uint8)


def _affine(img, m):
    """Nearest-neighbour inverse map m = (m0..m5) in centred coordinates, zero fill."""
    C, H, W = img.shape
    jj, ii = np.meshgrid(np.arange(H, dtype=f32), np.arange(W, dtype=f32), indexing="ij")
    X = ii - f32(W * 0.5) + f32(0.5)
    Y = jj - f32(H * 0.5) + f32(0.5)
    m0, m1, m2, m3, m4, m5 = (f32(v) for v in m)
    xs = m0 * X + m1 * Y + m2
    ys = m3 * X + m4 * Y + m5
    sx = np.rint(xs + f32(W * 0.5 - 0.5)).astype(np.int64)
    sy = np.rint(ys + f32(H * 0.5 - 0.5)).astype(np.int64)
    ok = (sx >= 0) & (sx < W) & (sy >= 0) & (sy < H)
    out = np.zeros_like(img)
    out[:, ok] = img[:, sy[ok], sx[ok]]
    return out


def affine_matrix(op: str, mag: float, H: int, W: int, cos_t=None, sin_t=None):
    """torchvision's inverse affine matrix for the op (see augment.hip)."""
    mag = f32(mag)
    if op == "ShearX":     # center [0, 0] -> centred (-W/2, -H/2)
        return (1.0, mag, mag * f32(H * 0.5), 0.0, 1.0, 0.0)
    if op == "ShearY":
        return (1.0, 0.0, 0.0, mag, 1.0, mag * f32(W * 0.5))
    if op == "TranslateX":
        return (1.0, 0.0, -float(int(mag)), 0.0, 1.0, 0.0)
    if op == "TranslateY":
        return (1.0, 0.0, 0.0, 0.0, 1.0, -float(int(mag)))
    if op == "Rotate":
        return (cos_t, sin_t, 0.0, -sin_t, cos_t, 0.0)
    raise ValueError(op)


def rotation_cs(angle_deg_f32):
    r = math.radians(-float(angle_deg_f32))
    return f32(math.cos(r)), f32(math.sin(r))


def _equalize_channel(ch):
    hist = np.bincount(ch.reshape(-1), minlength=256).astype(np.int64)
    nz = hist[hist != 0]
    step = int(nz[:-1].sum()) // 255
    if step == 0:
        return ch.copy()
    lut = (np.cumsum(hist) + step // 2) // step
    lut = np.concatenate([[0], lut[:-1]]).clip(0, 255)
    return lut[ch.astype(np.int64)].astype(np.uint8)


def apply_op(img: np.ndarray, op: str, mag: float) -> np.ndarray:
    """One op on a [C][H][W] uint8 image (mag already signed)."""
    C, H, W = img.shape
    if op == "Identity":
        return img.copy()
    if op in ("ShearX", "ShearY", "TranslateX", "TranslateY"):
        return _affine(img, affine_matrix(op, mag, H, W))
    if op == "Rotate":
        c, s = rotation_cs(mag)
        return _affine(img, affine_matrix(op, mag, H, W, c, s))
    if op == "Brightness":
        return _blend(img, np.zeros_like(img), mag)
    if op == "Color":   # adjust_saturation: a 1-channel image is returned unchanged
        return img.copy() if C == 1 else _blend(img, np.broadcast_to(_gray(img), img.shape), mag)
    if op == "Contrast":
        g = _gray(img).astype(np.int64)
        mean = f32(g.sum()) / f32(H * W)
        return _blend(img, np.full(img.shape, mean, f32), mag)
    if op == "Sharpness":
        deg = img.copy()
        x = img.astype(np.int64)
        s = (x[:, :-2, :-2] + x[:, :-2, 1:-1] + x[:, :-2, 2:] + x[:, 1:-1, :-2] + 5 * x[:, 1:-1, 1:-1] + x[:, 1:-1, 2:]
             + x[:, 2:, :-2] + x[:, 2:, 1:-1] + x[:, 2:, 2:])
        deg[:, 1:-1, 1:-1] = np.rint(s.astype(f32) / f32(13.0)).astype(np.uint8)
        return _blend(img, deg, mag)
    if op == "Posterize":
        bits = int(mag)
        mask = (0xFF << (8 - bits)) & 0xFF
        return img & np.uint8(mask)
    if op == "Solarize":
        return np.where(img.astype(f32) >= f32(mag), 255 - img, img).astype(np.uint8)
    if op == "AutoContrast":
        out = np.empty_like(img)
        for c in range(C):
            lo, hi = f32(img[c].min()), f32(img[c].max())
            if hi == lo:
                lo, scale = f32(0.0), f32(1.0)
            else:
                scale = f32(255.0) / (hi - lo)
            out[c] = np.clip((img[c].astype(f32) - lo) * scale, f32(0), f32(255)).astype(np.uint8)
        return out
    if op == "Equalize":
        return np.stack([_equalize_channel(img[c]) for c in range(C)])
    if op == "Invert":
        return (255 - img).astype(np.uint8)
    raise ValueError(op)


def signed_magnitude(op_id: int, bin_: int, sign_bit: int, mags: np.ndarray) -> float:
    if bin_ < 0:
        return 0.0
    m = float(mags[op_id, bin_])
    if OPS[op_id] in SIGNED and sign_bit == 0:
        m = -m
    return m


def augment_reference(images: np.ndarray, index: np.ndarray, seed: int, mode: int, pad: int = 4,
                      fixed=None) -> np.ndarray:
    """uint8 [B][C][H][W] batch exactly as the kernel augments it (before normalisation).
    ``fixed`` = (op id, bin, sign bit): apply only that op (the kernel's test hook)."""
    _, C, H, W = images.shape
    mags = magnitude_table(H, W)
    ops, prob, bins, _ = policy_table()
    out = np.empty((len(index), C, H, W), np.uint8)
    for b, row in enumerate(index):
        img = images[row].copy()
        d = draws(seed, b)
        if fixed is not None:
            op, bn, sg = fixed
            img = apply_op(img, OPS[op], signed_magnitude(op, bn, sg, mags))
        elif mode & MODE_AUTOAUGMENT:
            for i in range(2):
                k = 2 * d["policy"] + i
                if d["u"][i] <= prob[k]:
                    img = apply_op(img, OPS[ops[k]], signed_magnitude(ops[k], bins[k], d["sign"][i], mags))
        if mode & MODE_FLIP_CROP:
            if d["flip"]:
                img = img[:, :, ::-1]
            dy, dx = d["dy"] % (2 * pad + 1), d["dx"] % (2 * pad + 1)
            p = np.zeros((C, H + 2 * pad, W + 2 * pad), np.uint8)
            p[:, pad:pad + H, pad:pad + W] = img
            img = p[:, dy:dy + H, dx:dx + W]
        out[b] = img
    return out
