"""Data partitioners, vectorised over label arrays.

Reference behaviour kept (index ranges, class choice, top-up / trim order):
* balanced (IID): rank r gets the contiguous range
  [sum_{j<r} floor(T*rho_j), + floor(T*rho_r))            BAR/dataloader.py:53-75
* class-skewed: same range; "fixed classes" {2r, 2r+1} mod C are topped up
  (drawn with replacement from the whole set) to round(len*fixed_ratio) and
  random-class samples trimmed to keep the size; shuffled  DAR/dataloader.py:56-105
* dynamic re-partition every global epoch: n = floor(T*rho); keep
  floor(n*prev_fraction) sampled from the previous shard, add
  floor(n*next_fraction) from the complement; (skewed) replace non-fixed
  indices until the fixed-class count reaches (prev+next)*fixed_ratio
                                                           BAR/dataloader.py:77-104, DAR :107-155

Fixed: every draw uses an explicit seeded numpy Generator,
and the O(N^2) Python label scans (which decoded and augmented an image per
label lookup) become numpy mask operations on the label array.
"""
from __future__ import annotations

import numpy as np


def contiguous_range(total: int, ratios, rank: int) -> tuple[int, int]:
    start = 0
    for i, r in enumerate(ratios):
        n = int(total * r)
        if i == rank:
            return start, start + n
        start += n
    raise IndexError(f"rank {rank} out of range for {len(ratios)} ratios")


def balanced_partition(total: int, ratios, rank: int) -> np.ndarray:
    s, e = contiguous_range(total, ratios, rank)
    return np.arange(s, e, dtype=np.int64)


def fixed_classes_of(rank: int, num_classes: int = 10) -> list[int]:
    return [(rank * 2) % num_classes, (rank * 2 + 1) % num_classes]


def skewed_partition(labels: np.ndarray, ratios, rank: int, fixed_ratio: float, num_classes: int = 10,
                     rng: np.random.Generator | None = None) -> tuple[np.ndarray, list[int]]:
    rng = rng or np.random.default_rng(0)
    labels = np.asarray(labels)
    s, e = contiguous_range(len(labels), ratios, rank)
    fixed = fixed_classes_of(rank, num_classes)
    idx = np.arange(s, e, dtype=np.int64)
    is_fixed = np.isin(labels[idx], fixed)
    fixed_idx = idx[is_fixed]
    rand_idx = idx[~is_fixed]
    want = int(round((e - s) * fixed_ratio))
    if len(fixed_idx) < want:
        pool_mask = np.isin(labels, fixed)
        pool_mask[fixed_idx] = False
        pool = np.nonzero(pool_mask)[0]
        if len(pool):
            extra = rng.choice(pool, size=want - len(fixed_idx), replace=True)
            fixed_idx = np.concatenate([fixed_idx, extra])
    excess = len(fixed_idx) + len(rand_idx) - (e - s)
    if excess > 0:
        rand_idx = rand_idx[: len(rand_idx) - excess]
    out = np.concatenate([fixed_idx, rand_idx]).astype(np.int64)
    rng.shuffle(out)
    return out, fixed


def next_partition(total: int, prev_indices: np.ndarray, share: float, prev_fraction: float, next_fraction: float,
                   rng: np.random.Generator, replace: bool = False, labels: np.ndarray | None = None,
                   fixed_classes=None, fixed_ratio: float | None = None) -> np.ndarray:
    prev_indices = np.asarray(prev_indices, dtype=np.int64)
    n = int(total * share)
    n_prev = int(n * prev_fraction)
    n_next = int(n * next_fraction)
    if len(prev_indices) == 0:
        keep = np.zeros(0, dtype=np.int64)
    else:
        keep = rng.choice(prev_indices, size=min(n_prev, len(prev_indices)) if not replace else n_prev,
                          replace=replace)
    mask = np.ones(total, dtype=bool)
    mask[keep] = False
    rest = np.nonzero(mask)[0]
    add = rng.choice(rest, size=min(n_next, len(rest)) if not replace else n_next, replace=replace) if len(rest) else \
        np.zeros(0, dtype=np.int64)
    out = np.concatenate([keep, add]).astype(np.int64)
    if labels is not None and fixed_classes is not None and fixed_ratio is not None:
        labels = np.asarray(labels)
        want = int((n_prev + n_next) * fixed_ratio)
        is_fixed = np.isin(labels[out], fixed_classes)
        have = int(is_fixed.sum())
        if have < want:
            need = want - have
            pool_mask = np.isin(labels, fixed_classes)
            pool_mask[out] = False
            pool = np.nonzero(pool_mask)[0]
            replaceable = np.nonzero(~is_fixed)[0]
            if len(pool) and len(replaceable):
                need = min(need, len(replaceable))
                repl = rng.choice(pool, size=need, replace=True)
                # the reference pops from the end of the replaceable list
                out[replaceable[::-1][:need]] = repl
    rng.shuffle(out)
    return out


def shares_from_durations(durations, rule: str = "throughput") -> list[float]:
    """Per-rank data share from measured epoch/probe durations.

    'reference_duration': own / sum (the reference's rule -- a SLOWER worker gets
    MORE data); 'throughput': proportional to 1/duration (a faster worker gets
    more data, so all ranks finish together)."""
    d = np.asarray(durations, dtype=np.float64)
    d = np.where(d <= 0, d[d > 0].min() if (d > 0).any() else 1.0, d)
    if rule == "reference_duration":
        w = d
    elif rule == "throughput":
        w = 1.0 / d
    elif rule == "equal":
        w = np.ones_like(d)
    else:
        raise ValueError(rule)
    return (w / w.sum()).tolist()
