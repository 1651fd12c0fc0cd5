"""Datasets without torchvision.

* ``synthetic(kind, n)``: MNIST- / CIFAR- / ImageNet-shaped uint8 images with a
  learnable class structure (per-class prototype + noise), generated from a
  seed -- this container has no network, so benchmarks and tests run on these.
* ``load_cifar10(root)``: the CIFAR-10 *binary* format reader (data_batch_*.bin,
  test_batch.bin), used when the files exist locally; no download.
* ``channel_stats``: per-channel mean / std over a training set, as the
  reference computes before building its Normalize transform
  (BAR/dataloader.py:10-13).

Datasets are stored as uint8 tensors and normalised on the device in the
loader, which keeps a whole CIFAR-10 (150 MB) resident in HBM next to the model.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch

SHAPES = {
    "mnist": (1, 28, 28),
    "cifar10": (3, 32, 32),
    "imagenet": (3, 224, 224),
    "imagenet64": (3, 64, 64),
}
CLASSES = {"mnist": 10, "cifar10": 10, "imagenet": 1000, "imagenet64": 1000}


@dataclass
class ArrayDataset:
    images: torch.Tensor          # [N, C, H, W] uint8 (or float)
    labels: torch.Tensor          # [N] int64
    num_classes: int
    mean: tuple | None = None     # per-channel, in [0,1] units
    std: tuple | None = None
    name: str = ""

    def __len__(self):
        return int(self.labels.numel())

    def __getitem__(self, i):
        return self.images[i], int(self.labels[i])

    @property
    def targets(self) -> np.ndarray:
        return self.labels.cpu().numpy()

    @property
    def shape(self):
        return tuple(self.images.shape[1:])


def synthetic(kind: str = "cifar10", n: int = 50_000, num_classes: int | None = None, seed: int = 0,
              noise: float = 0.9, proto_seed: int | None = None, hard: bool = False) -> ArrayDataset:
    """Seeded, learnable synthetic images: x = clip(proto[y] + noise), uint8.
    `proto_seed` fixes the class prototypes (share it between train and test sets).

    ``hard`` (dataset names ``*-hard``): a task that does NOT saturate, so topology /
    skew effects show in the curves -- low-contrast overlapping prototypes (amplitude
    0.3 around grey), a random +-3 px shift and contrast jitter per image, and 15 %
    of the labels (train and test alike) redrawn uniformly, which caps the reachable
    test accuracy near 86 %."""
    shape = SHAPES[kind]
    k = num_classes or CLASSES[kind]
    g = torch.Generator().manual_seed(seed if proto_seed is None else proto_seed)
    # low-frequency class prototypes (upsampled 4x4 / 7x7 noise) so convs can learn them
    base = max(2, shape[1] // 8)
    protos = torch.rand(k, shape[0], base, base, generator=g)
    protos = torch.nn.functional.interpolate(protos, size=shape[1:], mode="bilinear", align_corners=False)
    if hard:
        protos = 0.5 + 0.3 * (protos - 0.5)
    gl = torch.Generator().manual_seed(seed + 1)
    labels = torch.randint(0, k, (n,), generator=gl)
    imgs = torch.empty((n, *shape), dtype=torch.uint8)
    chunk = 4096
    gn = torch.Generator().manual_seed(seed + 2)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        p = protos[labels[s:e]]
        if hard:
            sid = torch.randint(0, 49, (e - s,), generator=gn)   # per-image (dy, dx) in [-3, 3]^2
            p = p.clone()
            for q in range(49):
                sel = sid == q
                if sel.any():
                    p[sel] = torch.roll(p[sel], shifts=(q // 7 - 3, q % 7 - 3), dims=(2, 3))
            p = 0.5 + (p - 0.5) * (0.6 + 0.8 * torch.rand(e - s, 1, 1, 1, generator=gn))
        x = p + noise * torch.randn((e - s, *shape), generator=gn)
        imgs[s:e] = (x.clamp(0, 1) * 255).round().to(torch.uint8)
    if hard:
        flip = torch.rand(n, generator=gl) < 0.15
        labels = torch.where(flip, torch.randint(0, k, (n,), generator=gl), labels)
    return ArrayDataset(imgs, labels, k, name=f"synthetic-{kind}{'-hard' if hard else ''}")


def load_cifar10(root: str = "data") -> tuple[ArrayDataset, ArrayDataset] | None:
    """Read the CIFAR-10 binary distribution if present under root; else None."""
    d = os.path.join(root, "cifar-10-batches-bin")
    if not os.path.isdir(d):
        return None

    def read(files):
        xs, ys = [], []
        for f in files:
            raw = np.fromfile(os.path.join(d, f), dtype=np.uint8).reshape(-1, 3073)
            ys.append(raw[:, 0].astype(np.int64))
            xs.append(raw[:, 1:].reshape(-1, 3, 32, 32))
        return torch.from_numpy(np.concatenate(xs)), torch.from_numpy(np.concatenate(ys))

    tr = read([f"data_batch_{i}.bin" for i in range(1, 6)])
    te = read(["test_batch.bin"])
    return ArrayDataset(tr[0], tr[1], 10, name="cifar10"), ArrayDataset(te[0], te[1], 10, name="cifar10-test")


def channel_stats(ds: ArrayDataset) -> tuple[tuple, tuple]:
    """Per-channel mean/std in [0,1] units over the whole set (BAR/dataloader.py:10-13)."""
    x = ds.images
    c = x.shape[1]
    s = torch.zeros(c, dtype=torch.float64)
    ss = torch.zeros(c, dtype=torch.float64)
    cnt = 0
    for i in range(0, x.shape[0], 8192):
        b = x[i: i + 8192].to(torch.float64) / (255.0 if x.dtype == torch.uint8 else 1.0)
        s += b.sum(dim=(0, 2, 3))
        ss += (b * b).sum(dim=(0, 2, 3))
        cnt += b.shape[0] * b.shape[2] * b.shape[3]
    mean = s / cnt
    std = (ss / cnt - mean * mean).clamp_min(1e-12).sqrt()
    return tuple(mean.tolist()), tuple(std.tolist())


def random_split_indices(n: int, fractions=(0.8, 0.2), seed: int = 0) -> list[np.ndarray]:
    """Seeded split (the reference's random_split is unseeded per rank: SURVEY Q8)."""
    perm = np.random.default_rng(seed).permutation(n)
    out, s = [], 0
    for i, f in enumerate(fractions):
        e = n if i == len(fractions) - 1 else s + int(round(f * n))
        out.append(perm[s:e])
        s = e
    return out


def build_dataset(name: str, n_train: int | None = None, n_test: int | None = None, seed: int = 0,
                  root: str = "data") -> tuple[ArrayDataset, ArrayDataset]:
    """'cifar10' uses the real binary files when present, else synthetic of that shape."""
    if name == "cifar10" and n_train is None:
        real = load_cifar10(root)
        if real is not None:
            return real
    kind = name.replace("synthetic-", "")
    hard = kind.endswith("-hard")
    kind = kind[: -len("-hard")] if hard else kind
    ntr = n_train or {"mnist": 60_000, "cifar10": 50_000}.get(kind, 10_000)
    nte = n_test or max(1, ntr // 5)
    tr = synthetic(kind, ntr, seed=seed, proto_seed=seed, hard=hard)
    te = synthetic(kind, nte, seed=seed + 1000, proto_seed=seed, hard=hard)
    te.name = tr.name + "-test"
    return tr, te
