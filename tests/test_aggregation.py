"""Aggregation formulas on an in-process fake world (SURVEY §4 'aggregation math')."""
import copy

import pytest
import torch

from ldnn.models.mlp import mlp2
from ldnn.parallel import aggregation as A
from ldnn.parallel.comm import FakeWorld
from ldnn.utils.flat_params import FlatParams


def _vals(n, size=37, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(size, generator=g) for _ in range(n)]


@pytest.mark.parametrize("N", [1, 2, 3, 5])
@pytest.mark.parametrize("weighted", [False, True])
def test_allreduce_mix(N, weighted):
    xs = _vals(N)
    w = 0.7
    out = FakeWorld(N).run(lambda c: (lambda b: (A.allreduce_mix(b, c, weighted, w), b)[1])(xs[c.rank].clone()))
    S = sum(xs)
    for r in range(N):
        if N == 1:
            exp = xs[r]
        elif weighted:
            exp = w * xs[r] + (1 - w) * (S - xs[r]) / (N - 1)
        else:
            exp = S / N
        torch.testing.assert_close(out[r], exp, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("N", [2, 3, 5])
@pytest.mark.parametrize("hops", [1, 2])
@pytest.mark.parametrize("weighted", [False, True])
def test_gossip_formulas(N, hops, weighted):
    xs = _vals(N, seed=1)
    w = 0.6

    def body(c):
        b = xs[c.rank].clone()
        A.gossip_mix(b, c, hops, weighted, w)
        return b

    out = FakeWorld(N).run(body)
    for r in range(N):
        x, y1, y2 = xs[r], xs[(r - 1) % N], xs[(r - 2) % N]
        if hops == 1:
            exp = w * x + (1 - w) * y1 if weighted else (x + y1) / 2
        else:
            exp = w * x + (1 - w) / 2 * (y1 + y2) if weighted else (x + y1 + y2) / 3
        torch.testing.assert_close(out[r], exp, rtol=1e-5, atol=1e-6)


def test_equal_ring_gossip_converges_to_mean():
    N = 4
    xs = _vals(N, seed=2)

    def body(c):
        b = xs[c.rank].clone()
        for _ in range(200):
            A.gossip_mix(b, c, 1, False, 0.5)
        return b

    out = FakeWorld(N).run(body)
    mean = sum(xs) / N
    for o in out:
        torch.testing.assert_close(o, mean, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("by", ["gradients", "weights"])
@pytest.mark.parametrize("topology", ["allreduce", "ring", "double_ring"])
def test_aggregator_on_models_matches_tensor_math(by, topology):
    N = 3
    torch.manual_seed(0)
    models = [mlp2(784, 16, 10) for _ in range(N)]
    for m in models:
        FlatParams(m, "cpu")
        for p in m.parameters():
            p.grad.copy_(torch.randn_like(p))
    before = [copy.deepcopy([(p.detach().clone(), p.grad.detach().clone()) for p in m.parameters()]) for m in models]

    def body(c):
        A.Aggregator(topology, "equal", by, comm=c)(models[c.rank])
        return [(p.detach().clone(), p.grad.detach().clone()) for p in models[c.rank].parameters()]

    out = FakeWorld(N).run(body)
    k = 0 if by == "weights" else 1
    for r in range(N):
        for t in range(len(before[r])):
            x = [before[q][t][k] for q in range(N)]
            if topology == "allreduce":
                exp = sum(x) / N
            elif topology == "ring":
                exp = (x[r] + x[(r - 1) % N]) / 2
            else:
                exp = (x[r] + x[(r - 1) % N] + x[(r - 2) % N]) / 3
            torch.testing.assert_close(out[r][t][k], exp, rtol=1e-5, atol=1e-6)
            # the other target is untouched
            torch.testing.assert_close(out[r][t][1 - k], before[r][t][1 - k])


def test_reference_named_functions():
    N = 2
    xs = _vals(N, seed=4)

    def body(c):
        b = xs[c.rank].clone()
        A.ring_all_reduce_weighted(b, c.rank, N, 0.8, comm=c)
        d = xs[c.rank].clone()
        A.double_ring_all_reduce(d, c.rank, N, comm=c)
        return b, d

    out = FakeWorld(N).run(body)
    torch.testing.assert_close(out[0][0], 0.8 * xs[0] + 0.2 * xs[1])
    # N=2: the 2-hop neighbour is the rank itself
    torch.testing.assert_close(out[0][1], (xs[0] + xs[1] + xs[0]) / 3)


def test_check_schedule_raises_on_every_rank_when_one_rank_reports_a_collective_error():
    """a one-shot IPC timeout is usually recorded on the late rank only.
    check_schedule gathers every rank's error flag with the schedule digest, so EVERY
    rank raises the same RuntimeError at the same point (none is left waiting in the
    next collective until the process-group timeout)."""
    from ldnn.parallel.comm import FakeComm, RankDivergenceError

    class _ErrComm(FakeComm):
        def local_error(self):
            return "one-shot all-reduce timed out" if self.rank == 1 else None

    world = FakeWorld(3, timeout=10)

    def body(c):
        c.__class__ = _ErrComm
        c.all_reduce(torch.ones(4))
        try:
            c.check_schedule("step 7")
        except RankDivergenceError:
            return "divergence"
        except RuntimeError as e:
            return str(e)
        return "ok"

    got = world.run(body)
    assert all(g.startswith("collective failure on rank(s) [1] at step 7") for g in got), got
    assert "timed out" in got[1]
