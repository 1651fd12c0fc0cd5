"""Device-resident data loading + the reference's loader factory API.

The reference feeds the GPU from a CPU DataLoader (num_workers=0, PIL
AutoAugment, per-batch H2D copies: SURVEY Q9, BAR/dataloader.py:16,42).  On a
288 GB MI355X the whole dataset fits in HBM many times over, so
``DeviceLoader`` keeps the uint8 images resident on the device and builds each
batch with an on-device gather + fused normalise + cast; nothing crosses PCIe
per step.  ``get_loaders`` / ``get_subset_loaders`` / ``estimate_epoch_duration``
keep the reference's signatures and return tuples (BAR/dataloader.py:9-153,
DAR/dataloader.py:9-204).
"""
from __future__ import annotations

import time

import numpy as np
import torch

from ..ops import _ext
from . import autoaugment as AA
from . import partition as P
from .datasets import ArrayDataset, build_dataset, channel_stats, random_split_indices

_RESIDENT: dict = {}


def _resident(t: torch.Tensor, device) -> torch.Tensor:
    device = torch.device(device)
    if t.device == device:
        return t
    key = (t.data_ptr(), tuple(t.shape), t.dtype, str(device))
    r = _RESIDENT.get(key)
    if r is None:
        r = t.to(device, non_blocking=False)
        _RESIDENT[key] = r
    return r


AUGMENT_MODES = {"none": 0, "autoaugment": AA.MODE_AUTOAUGMENT, "flipcrop": AA.MODE_FLIP_CROP,
                 "autoaugment+flipcrop": AA.MODE_AUTOAUGMENT | AA.MODE_FLIP_CROP}


def augment_mode(augment) -> int:
    """False/None/'none' -> 0; True/'autoaugment' -> AutoAugment(CIFAR10) (the reference's
    train transform, BAR/dataloader.py:16); 'flipcrop'; 'autoaugment+flipcrop'."""
    if augment is None or augment is False:
        return 0
    if augment is True:
        return AA.MODE_AUTOAUGMENT
    if augment not in AUGMENT_MODES:
        raise ValueError(f"augment must be one of {sorted(AUGMENT_MODES)}, got {augment!r}")
    return AUGMENT_MODES[augment]


class DeviceLoader:
    """Batches of (normalised image, label) gathered on the device.

    ``indices`` select rows of ``dataset`` (a shard); iteration order is the
    shard order (shuffle=False, as in the reference) or a seeded per-epoch
    permutation.  On a GPU with a uint8 dataset each batch is ONE native launch
    (augment.hip): gather + optional AutoAugment / flip+crop + normalise + cast.
    The augmentation draws are counter hashes of (seed, epoch, batch, sample):
    reproducible, and identical on the CPU path (data/autoaugment.py)."""

    def __init__(self, dataset: ArrayDataset, indices, batch_size: int, device, shuffle: bool = False,
                 drop_last: bool = False, seed: int = 0, mean=None, std=None, dtype=torch.float32,
                 augment=False, pad: int = 4):
        self.dataset = dataset
        self.device = torch.device(device)
        self.batch_size = int(batch_size)
        self.shuffle, self.drop_last = shuffle, drop_last
        self.dtype = dtype
        self.augment = augment
        self.mode = augment_mode(augment)
        self.pad = int(pad)
        self.images = _resident(dataset.images, self.device)
        self.labels = _resident(dataset.labels, self.device)
        idx = np.arange(len(dataset)) if indices is None else np.asarray(indices, dtype=np.int64)
        if idx.size and (idx.min() < 0 or idx.max() >= len(dataset)):
            raise IndexError(f"shard indices outside [0, {len(dataset)})")
        self.indices_np = idx
        self.indices = torch.as_tensor(idx, dtype=torch.long, device=self.device)
        mean = mean if mean is not None else dataset.mean
        std = std if std is not None else dataset.std
        c = dataset.images.shape[1]
        scale = 255.0 if dataset.images.dtype == torch.uint8 else 1.0
        m = torch.tensor(mean if mean is not None else [0.0] * c, dtype=torch.float32, device=self.device)
        s = torch.tensor(std if std is not None else [1.0] * c, dtype=torch.float32, device=self.device)
        # x_norm = x_raw * a + b  (fused into one multiply-add on the device)
        self._a = (1.0 / (scale * s)).view(1, c, 1, 1)
        self._b = (-m / s).view(1, c, 1, 1)
        self._gen = torch.Generator().manual_seed(seed)
        self.seed = int(seed)
        self.epoch = 0
        self._native = (self.device.type == "cuda" and self.images.dtype == torch.uint8
                        and self.dtype in (torch.bfloat16, torch.float32) and _ext.use_native(self.images)
                        and c * dataset.images.shape[2] * dataset.images.shape[3] <= AA_MAX_PIXELS)
        if self.mode and self.images.dtype != torch.uint8:
            raise ValueError("augmentation needs a uint8 dataset")

    def __len__(self):
        n = len(self.indices_np)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    @property
    def num_samples(self) -> int:
        n = len(self.indices_np)
        return (n // self.batch_size) * self.batch_size if self.drop_last else n

    def _batch(self, idx: torch.Tensor, seed: int = 0):
        if self._native:
            _, C, H, W = self.images.shape
            out = torch.empty(idx.numel(), C, H, W, dtype=self.dtype, device=self.device)
            augment_native(self.images, idx, out, self._a.reshape(-1), self._b.reshape(-1), seed, self.mode, self.pad)
            return out, self.labels.index_select(0, idx)
        if self.mode:   # CPU (or non-native) path: the kernel's NumPy reference, same draws
            raw = AA.augment_reference(self.images.cpu().numpy(), idx.cpu().numpy(), seed, self.mode, self.pad)
            x = torch.from_numpy(raw).to(self.device)
        else:
            x = self.images.index_select(0, idx)
        x = torch.addcmul(self._b, x.to(torch.float32), self._a)
        return x.to(self.dtype), self.labels.index_select(0, idx)

    def __iter__(self):
        order = self.indices
        if self.shuffle:
            perm = torch.randperm(len(order), generator=self._gen).to(self.device)
            order = order[perm]
        epoch = self.epoch
        self.epoch += 1
        bs = self.batch_size
        n = len(order)
        end = (n // bs) * bs if self.drop_last else n
        for k, s in enumerate(range(0, end, bs)):
            yield self._batch(order[s: s + bs], AA.batch_seed(self.seed, epoch, k) if self.mode else 0)


AA_MAX_PIXELS = 28 * 1024   # csrc kAugMaxPixels
_AA_TABLES: dict = {}


def _aa_tables(H: int, W: int):
    t = _AA_TABLES.get((H, W))
    if t is None:
        mags = AA.magnitude_table(H, W)
        rc, rs = zip(*[AA.rotation_cs(v) for v in mags[AA.OP["Rotate"]]])
        ops, prob, bins, signed = AA.policy_table()
        t = ([float(v) for v in mags.reshape(-1)], [float(v) for v in rc], [float(v) for v in rs],
             [int(v) for v in ops], [float(v) for v in prob], [int(v) for v in bins], [int(v) for v in signed])
        _AA_TABLES[(H, W)] = t
    return t


def augment_native(images, idx, out, a, b, seed: int, mode: int, pad: int = 4, fixed=None):
    """One augment.hip launch: out = normalise(augment(images[idx])).  ``fixed`` =
    (op id, magnitude bin, sign bit) applies just that op (kernel test hook)."""
    H, W = images.shape[2], images.shape[3]
    fo, fb, fs = fixed if fixed is not None else (-1, 0, 0)
    _ext.C().augment_batch(images, idx, out, a.contiguous(), b.contiguous(), int(seed), int(mode), int(pad),
                           int(fo), int(fb), int(fs), *_aa_tables(H, W))
    return out


# ---------------------------------------------------------------- probe (A12)
def estimate_epoch_duration(trainloader, world_size, model, device, num_batches: int = 10, comm=None,
                            rule: str = "reference_duration"):
    """Time a few forward/backward passes and all-gather the durations.

    Returns (own_share, shares) like BAR/dataloader.py:119-153.  Fixes SURVEY
    Q12: BN running statistics and gradients are restored afterwards, and the
    device is synchronised so GPU time is actually measured."""
    from ..parallel.comm import default_comm

    from ..parallel.ddp import DataParallel

    comm = comm or default_comm()
    if isinstance(model, DataParallel):   # time the replica's own step: no gradient collectives
        model = model.module
    dev = torch.device(device)
    bn_state = {k: v.clone() for k, v in model.state_dict().items() if "running" in k or "num_batches" in k}
    was_training = model.training
    model.train()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i, (x, y) in enumerate(trainloader):
        if i >= num_batches:
            break
        out = model(x)
        out.float().sum().backward()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dur = time.perf_counter() - t0
    with torch.no_grad():
        for p in model.parameters():
            if p.grad is not None:
                p.grad.zero_()
        sd = model.state_dict()
        for k, v in bn_state.items():
            sd[k].copy_(v)
    model.train(was_training)
    t = torch.tensor([dur], dtype=torch.float32, device=dev)
    durs = [float(v.item()) for v in comm.all_gather(t)] if comm.world_size > 1 else [dur]
    shares = P.shares_from_durations(durs, rule)
    return shares[comm.rank], shares


# --------------------------------------------------------- reference factory
def get_loaders(batch_size, world_size, rank, model, device, fixed_ratio=None, *, dataset: str = "cifar10",
                comm=None, seed: int = 0, val_fraction: float = 0.2, partition_rule: str = "reference_duration",
                probe_batches: int = 10, n_train: int | None = None, n_test: int | None = None,
                dtype=torch.float32, augment=False, data_root: str = "data", augment_val: bool = False):
    """Build (train, val, test) loaders for this rank (BAR/dataloader.py:9-51).

    Returns the reference's 7-tuple (IID) or 8-tuple (+fixed_classes) when
    ``fixed_ratio`` is given (class-skewed, DAR/dataloader.py:9-52)."""
    full, testset = build_dataset(dataset, n_train, n_test, seed=seed, root=data_root)
    mean, std = channel_stats(full)
    full.mean, full.std = mean, std
    testset.mean, testset.std = mean, std
    tr_idx, va_idx = random_split_indices(len(full), (1.0 - val_fraction, val_fraction), seed=seed)
    trainset = ArrayDataset(full.images[torch.as_tensor(tr_idx)], full.labels[torch.as_tensor(tr_idx)],
                            full.num_classes, mean, std, full.name + "-train")
    valset = ArrayDataset(full.images[torch.as_tensor(va_idx)], full.labels[torch.as_tensor(va_idx)],
                          full.num_classes, mean, std, full.name + "-val")

    if partition_rule == "equal" or world_size == 1:
        shares = [1.0 / world_size] * world_size
    else:
        tmp = DeviceLoader(trainset, None, batch_size, device, shuffle=True, seed=seed + 17, dtype=dtype)
        _, shares = estimate_epoch_duration(tmp, world_size, model, device, probe_batches, comm, partition_rule)
    rng = np.random.default_rng(seed * 1009 + rank)
    if fixed_ratio is None:
        train_indices = P.balanced_partition(len(trainset), shares, rank)
        val_indices = P.balanced_partition(len(valset), shares, rank)
        fixed = None
    else:
        train_indices, fixed = P.skewed_partition(trainset.targets, shares, rank, fixed_ratio,
                                                  trainset.num_classes, rng)
        val_indices, _ = P.skewed_partition(valset.targets, shares, rank, fixed_ratio, valset.num_classes, rng)
    train_loader = DeviceLoader(trainset, train_indices, batch_size, device, dtype=dtype, augment=augment,
                                seed=(seed * 1_000_003 + rank * 10_007) & 0x7FFFFFFF)
    val_loader = DeviceLoader(valset, val_indices, batch_size, device, dtype=dtype,
                              augment=augment if augment_val else False, seed=(seed * 7 + rank * 13 + 5) & 0x7FFFFFFF)
    test_loader = DeviceLoader(testset, None, batch_size, device, dtype=dtype)
    out = (train_loader, val_loader, test_loader, trainset, valset, train_indices, val_indices)
    return out + (fixed,) if fixed_ratio is not None else out


def get_subset_loaders(trainset, valset, train_indices, val_indices, batch_size, prev_fraction, next_fraction,
                       share, device, rng: np.random.Generator, replace: bool = False, fixed_classes=None,
                       fixed_ratio=None, dtype=torch.float32, augment=False, loader_seed: int = 0,
                       augment_val: bool = False):
    """Re-partition for the next global epoch (BAR/dataloader.py:107-117)."""
    kw = {}
    if fixed_classes is not None:
        kw = dict(fixed_classes=fixed_classes, fixed_ratio=fixed_ratio)
    tr = P.next_partition(len(trainset), train_indices, share, prev_fraction, next_fraction, rng, replace,
                          labels=trainset.targets if kw else None, **kw)
    va = P.next_partition(len(valset), val_indices, share, prev_fraction, next_fraction, rng, replace,
                          labels=valset.targets if kw else None, **kw)
    return (DeviceLoader(trainset, tr, batch_size, device, dtype=dtype, augment=augment, seed=loader_seed),
            DeviceLoader(valset, va, batch_size, device, dtype=dtype, augment=augment if augment_val else False,
                         seed=(loader_seed * 31 + 7) & 0x7FFFFFFF), tr, va)
