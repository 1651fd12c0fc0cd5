"""train_global end-to-end on an in-process fake world: the 12-history contract,
every topology / target / weighting, the straggler cutoff, evaluation metrics."""
import numpy as np
import pytest
import torch

import ldnn
from ldnn.data.loader import get_loaders
from ldnn.models import CrossEntropyLoss, xavier_init
from ldnn.models.mlp import mlp2
from ldnn.optim import Adam, StepLR
from ldnn.parallel.comm import FakeWorld
from ldnn.train import straggler as S
from ldnn.train.trainer import train_global
from ldnn.train.validator import classification_report, evaluate


def _run_rank(comm, El=2, Eg=2, fixed_ratio=None, topology="allreduce", by="gradients", agg="equal",
              sync_every="global_epoch", timelimit=float("inf"), check_every=5, slow_rank=None, shrink_rank=None):
    torch.manual_seed(0)
    model = mlp2(784, 32, 10)
    xavier_init(model)
    flat = ldnn.prepare(model, "cpu")
    comm.broadcast(flat.master, 0)  # reference A6: replicas start identical
    loaders = get_loaders(32, comm.world_size, comm.rank, model, "cpu", fixed_ratio, dataset="mnist", comm=comm,
                          n_train=1200, n_test=200, partition_rule="equal")
    tr, va, te, trainset, valset, ti, vi = loaders[:7]
    fixed = loaders[7] if len(loaders) > 7 else None
    if shrink_rank is not None and comm.rank == shrink_rank:  # unequal shards: this rank finishes first
        from ldnn.data.loader import DeviceLoader

        ti = ti[: len(ti) // 4]
        tr = DeviceLoader(trainset, ti, 32, "cpu")
    crit = CrossEntropyLoss()
    opt = Adam(model.parameters(), lr=1e-3)
    if slow_rank is not None and comm.rank == slow_rank:
        orig = opt.step

        def slow_step(self, *a, **k):
            import time

            time.sleep(0.05)
            return orig(*a, **k)

        import types

        # a bound method, set before the scheduler wraps step (no scheduler-order warning)
        opt.step = types.MethodType(slow_step, opt)
    sch = StepLR(opt, step_size=25)
    H = train_global(model, tr, va, trainset, valset, ti, vi, crit, opt, sch, "cpu", comm.rank, comm.world_size, El,
                     Eg, timelimit, 32, 0.5, 0.5, 0.5, agg, by, comm=comm, topology=topology, fixed_classes=fixed,
                     fixed_ratio=fixed_ratio, sync_every=sync_every, progress=False, verbose=False,
                     check_every=check_every)
    return H, model, comm.schedule_digest()


@pytest.mark.parametrize("topology", ["allreduce", "ring", "double_ring"])
@pytest.mark.parametrize("by", ["gradients", "weights"])
def test_twelve_history_contract(topology, by):
    N, El, Eg = 3, 2, 2
    res = FakeWorld(N).run(_run_rank, El=El, Eg=Eg, topology=topology, by=by, agg="weighted")
    H0 = res[0][0]
    assert len(H0) == 12
    awl, ael, gel, gea, gtl, gta, gvl, gva, wtl, wta, wvl, wva = H0
    assert len(awl) == N and all(len(w) > 0 for w in awl)
    assert len(ael) == Eg * El
    assert len(gel) == Eg and len(gea) == Eg and all(len(a) == El for a in gea)
    for h in (gtl, gta, gvl, gva):
        assert len(h) == Eg
    for h in (wtl, wta, wvl, wva):
        assert len(h) == Eg * El
    # histories 5-8 are identical on every rank; collective schedules identical everywhere
    for r in range(1, N):
        assert res[r][0][4:8] == H0[4:8]
        assert res[r][2] == res[0][2]
    # the model learns something
    assert gta[-1] > 30.0
    if by == "weights" and topology == "allreduce":
        # equal... here weighted averaging with w=0.5 on N=3 still differs; replicas stay finite
        for _, m, _ in res:
            assert all(torch.isfinite(p).all() for p in m.parameters())


def test_weights_equal_allreduce_makes_replicas_identical():
    res = FakeWorld(3).run(_run_rank, El=1, Eg=1, by="weights", agg="equal")
    ps = [torch.cat([p.detach().flatten() for p in m.parameters()]) for _, m, _ in res]
    for p in ps[1:]:
        torch.testing.assert_close(p, ps[0])


def test_step_sync_keeps_replicas_identical():
    res = FakeWorld(2).run(_run_rank, El=1, Eg=1, sync_every="step", by="gradients")
    ps = [torch.cat([p.detach().flatten() for p in m.parameters()]) for _, m, _ in res]
    torch.testing.assert_close(ps[0], ps[1])


def test_skewed_partition_training():
    res = FakeWorld(2).run(_run_rank, El=1, Eg=2, fixed_ratio=0.5)
    assert len(res[0][0][4]) == 2


def test_straggler_cutoff_fires_collectively():
    # rank 1 is slow; a 0.2 s limit after rank 0 finishes cuts rank 1's local epochs short
    res = FakeWorld(2).run(_run_rank, El=3, Eg=1, timelimit=0.2, check_every=2, slow_rank=1, shrink_rank=0)
    wtl = res[0][0][8]
    assert len(wtl) == 3  # rank 0 completed its 3 local epochs
    awl = res[0][0][0]
    assert len(awl[0]) == 3 * 4  # rank 0: 3 local epochs of its small shard
    assert len(awl[1]) < 3 * 15  # rank 1 (15 batches / epoch) was cut short
    assert res[0][2] == res[1][2]  # same collective schedule on both ranks


def test_cutoff_unit_rounds():
    w = FakeWorld(2)

    def body(c):
        cut = S.StragglerCutoff(c, 0.0, check_every=1)
        steps = 0
        try:
            for i in range(1000):
                if c.rank == 0 and i == 3:
                    break
                steps += 1
                cut.step(i)
        except S.StopLocalTraining:
            pass
        cut.finish()
        return steps

    s0, s1 = w.run(body)
    assert s0 == 3 and s1 < 1000


def test_classification_report_matches_sklearn():
    from sklearn.metrics import precision_recall_fscore_support

    rng = np.random.default_rng(0)
    y = rng.integers(0, 7, 500)
    p = np.where(rng.random(500) < 0.6, y, rng.integers(0, 7, 500))
    p[p == 6] = 5  # a class never predicted
    rep = classification_report(torch.from_numpy(p), torch.from_numpy(y), 7)
    for avg in ("macro", "weighted", "micro"):
        pr, rc, f1, _ = precision_recall_fscore_support(y, p, average=avg, zero_division=0)
        assert abs(rep["precision_" + avg] - pr) < 1e-9
        assert abs(rep["recall_" + avg] - rc) < 1e-9
        assert abs(rep["f1_" + avg] - f1) < 1e-9


def test_evaluate_returns_reference_tuple():
    torch.manual_seed(0)
    m = mlp2(784, 16, 10)
    ldnn.prepare(m, "cpu")
    from ldnn.data.datasets import synthetic
    from ldnn.data.loader import DeviceLoader

    ds = synthetic("mnist", 256, seed=1)
    loss, acc, preds, labels = evaluate(m, DeviceLoader(ds, None, 64, "cpu"), CrossEntropyLoss(), "cpu", 0,
                                        num_classes=10, verbose=False)
    assert preds.shape == labels.shape == (256,)
    assert 0 <= acc <= 100 and loss > 0
