"""Partitioners (SURVEY §4 'partitioners' row; reference A13-A16)."""
import numpy as np
import pytest

from ldnn.data import partition as P


def test_balanced_ranges_match_reference_rule():
    T, ratios = 40_000, [0.2] * 5
    parts = [P.balanced_partition(T, ratios, r) for r in range(5)]
    assert [len(p) for p in parts] == [8000] * 5
    assert parts[0][0] == 0 and parts[4][-1] == T - 1
    assert len(np.unique(np.concatenate(parts))) == T
    # floor(T*rho) per rank, contiguous
    ratios = [0.1, 0.3, 0.6]
    s, e = P.contiguous_range(1001, ratios, 2)
    assert (s, e) == (int(1001 * 0.1) + int(1001 * 0.3), int(1001 * 0.1) + int(1001 * 0.3) + int(1001 * 0.6))


@pytest.mark.parametrize("rank", [0, 1, 4, 6])
def test_skewed_partition_fixed_fraction(rank):
    rng = np.random.default_rng(0)
    labels = rng.integers(0, 10, size=20_000)
    idx, fixed = P.skewed_partition(labels, [0.1] * 10, rank, 0.5, 10, np.random.default_rng(1))
    assert fixed == [(2 * rank) % 10, (2 * rank + 1) % 10]
    assert len(idx) == 2000
    frac = np.isin(labels[idx], fixed).mean()
    assert frac >= 0.5 - 1e-9
    # seeded -> reproducible
    idx2, _ = P.skewed_partition(labels, [0.1] * 10, rank, 0.5, 10, np.random.default_rng(1))
    assert np.array_equal(idx, idx2)


def test_next_partition_fractions_and_disjointness():
    rng = np.random.default_rng(3)
    prev = np.arange(0, 2000)
    out = P.next_partition(10_000, prev, 0.25, 0.5, 0.5, rng, replace=False)
    assert len(out) == int(int(10_000 * 0.25) * 0.5) * 2
    n_prev = np.isin(out, prev).sum()
    assert n_prev >= int(2500 * 0.5)  # kept part comes from prev
    assert len(np.unique(out)) == len(out)  # replace=False -> no duplicates


def test_next_partition_skewed_topup():
    rng = np.random.default_rng(5)
    labels = np.random.default_rng(9).integers(0, 10, 10_000)
    prev = np.arange(1000)
    out = P.next_partition(10_000, prev, 0.2, 0.5, 0.5, rng, replace=True, labels=labels, fixed_classes=[0, 1],
                           fixed_ratio=0.6)
    assert np.isin(labels[out], [0, 1]).mean() >= 0.6 - 1e-9


def test_share_rules():
    d = [1.0, 2.0, 4.0]
    ref = P.shares_from_durations(d, "reference_duration")
    thr = P.shares_from_durations(d, "throughput")
    assert np.allclose(ref, [1 / 7, 2 / 7, 4 / 7])  # reference: slower worker gets MORE data (Q6)
    assert thr[0] > thr[1] > thr[2]  # throughput rule: faster worker gets more
    assert abs(sum(thr) - 1) < 1e-12
