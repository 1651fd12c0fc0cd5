"""DataParallel(shard_optimizer=True): reduce-scatter + sharded fused optimizer + weight
all-gather (parallel/ddp.py) == the all-reduce + replicated optimizer path, on CPU.

FakeWorld (threads) pins the math for SGD-momentum, Adam and the reference's weighted
all-reduce (BAR/communication.py:4-10) on a conv net (LeNet-5: conv + Linear weights and
biases) and a BatchNorm net (the reference's small EnhancedCNN variant); a gloo
2-process run drives the same path through the CLI (train.py --sync_every step)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

import ldnn
from ldnn.models import CrossEntropyLoss, build_model, xavier_init
from ldnn.optim import SGD, Adam
from ldnn.parallel.comm import FakeWorld
from ldnn.parallel.ddp import DataParallel

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = {"lenet5": (1, 28, 28), "enhanced_cnn_small": (3, 32, 32)}


def _init_states():
    out = {}
    for nm in SHAPES:   # built once outside the rank threads: the global RNG is shared
        torch.manual_seed(0)
        m = build_model(nm)
        xavier_init(m)
        out[nm] = m.state_dict()
    return out


INIT = _init_states()


def _train(comm, name, shard, optname, local_weight=None, steps=3, batch=6):
    m = build_model(name)
    m.load_state_dict(INIT[name])
    ldnn.prepare(m, "cpu")
    dp = DataParallel(m, comm, bucket_cap_mb=0.05, shard_optimizer=shard, local_weight=local_weight)
    opt = SGD(m.parameters(), lr=0.05, momentum=0.9) if optname == "sgd" else Adam(m.parameters(), lr=1e-3)
    g = torch.Generator().manual_seed(10 + comm.rank)
    crit = CrossEntropyLoss()
    for _ in range(steps):
        x = torch.randn(batch, *SHAPES[name], generator=g)
        y = torch.randint(0, 10, (batch,), generator=g)
        opt.zero_grad()
        crit(dp(x), y).backward()
        dp.finish_gradient_sync()
        opt.step()
    dp.gather_master(opt)
    st = {k: v.clone() for k, v in m.state_dict().items()}
    f = dp.flat
    ost = {k: {s.name: f.storage_view(s, v).clone() for s in f.segments}
           for k, v in opt._ls().items() if torch.is_tensor(v) and v.shape == f.master.shape}
    return [b["sharded"] for b in dp.bucketer.buckets], st, ost


@pytest.mark.parametrize("name,optname,lw", [("lenet5", "sgd", None), ("lenet5", "adam", None),
                                             ("enhanced_cnn_small", "adam", None)])
def test_sharded_step_equals_allreduce_step(name, optname, lw):
    N = 3
    sh = FakeWorld(N).run(_train, name, True, optname, lw)
    ref = FakeWorld(N).run(_train, name, False, optname, lw)
    kinds = sh[0][0]
    assert kinds[-1] is False and sum(kinds) >= 2, kinds   # several reduce-scattered buckets + replicated tail
    for r in range(N):
        for k, v in ref[r][1].items():
            torch.testing.assert_close(sh[r][1][k].float(), v.float(), rtol=1e-5, atol=1e-6, msg=k)
    # the whole optimizer state is gathered too (momentum / Adam moments)
    assert set(ref[0][2]) == set(sh[0][2]) and ref[0][2]
    for r in range(N):
        for k, per in ref[r][2].items():
            for pn, v in per.items():   # per parameter: the two layouts differ
                torch.testing.assert_close(sh[r][2][k][pn], v, rtol=1e-5, atol=1e-7, msg=f"{k} {pn}")


def test_sharded_refuses_weighted_mix():
    """The reference's weighted all-reduce gives every rank its own update (replicas
    drift apart): no rank can own a shard of another's, so the combination is refused."""
    m = build_model("lenet5")
    ldnn.prepare(m, "cpu")
    with pytest.raises(ValueError, match="equal averaging"):
        DataParallel(m, FakeWorld(1).comm(0), shard_optimizer=True, local_weight=0.7)


def test_sharded_layout_alignment_and_ownership():
    """Every sharded bucket splits into N 256-B aligned shards, the ranks' update ranges
    tile the buffer exactly once (sharded) / N times (replicated tail), and the tail
    holds exactly the 1-D parameters."""
    N = 3
    torch.manual_seed(0)
    m = build_model("enhanced_cnn_small")
    ldnn.prepare(m, "cpu")

    def body(c):
        dp = DataParallel(m if c.rank == 0 else _clone(m), c, bucket_cap_mb=0.5, shard_optimizer=True,
                          broadcast_init=False)
        return dp.bucketer.update_ranges(), [(b["begin"], b["end"], b["sharded"], [p.dim() for p in b["params"]])
                                             for b in dp.bucketer.buckets], dp.flat.numel

    res = FakeWorld(N).run(body)
    buckets, numel = res[0][1], res[0][2]
    cover = torch.zeros(numel, dtype=torch.int32)
    for ranges, _, _ in res:
        for lo, hi in ranges:
            assert lo % 64 == 0
            cover[lo:hi] += 1
    for b, e, sharded, dims in buckets:
        assert (e - b) % (N * 64) == 0 or not sharded
        assert (cover[b:e] == (1 if sharded else N)).all()
        assert all(d >= 2 for d in dims) if sharded else all(d < 2 for d in dims)


def _clone(m):
    c = build_model("enhanced_cnn_small")
    c.load_state_dict(m.state_dict())
    ldnn.prepare(c, "cpu")
    return c


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.slow
def test_cli_sharded_per_step_dp_two_ranks(tmp_path):
    """train.py --sync_every step --shard_optimizer on, 2 gloo ranks: trains, checkpoints
    (gather_master before the rank-0 write) and ends with identical replicas."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(_port()), os.path.join(ROOT, "train.py"), "--model", "lenet5", "--dataset", "mnist",
           "--n_train", "600", "--n_test", "100", "--epochs_global", "2", "--epochs_local", "1", "--device", "cpu",
           "--quiet", "--out_dir", str(tmp_path), "--plots", "", "--sync_every", "step", "--shard_optimizer", "on",
           "--optimizer", "adam", "--checkpoint_every", "1", "--no_eval", "--bucket_mb", "0.05"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    ck = sorted((tmp_path / "ckpt").glob("ckpt_ge*.pt"))
    assert ck, list(tmp_path.iterdir())
    sd = torch.load(ck[-1], weights_only=True)
    assert "features.0.weight" in sd["model"] and sd["global_epoch"] == 2


def _two_groups(comm):
    m = build_model("lenet5")
    m.load_state_dict(INIT["lenet5"])
    ldnn.prepare(m, "cpu")
    dp = DataParallel(m, comm, bucket_cap_mb=0.05, shard_optimizer=True)
    ps = list(m.parameters())
    opt = SGD([{"params": ps[:2]}, {"params": ps[2:]}], lr=0.05)
    x = torch.randn(4, *SHAPES["lenet5"])
    y = torch.randint(0, 10, (4,))
    CrossEntropyLoss()(dp(x), y).backward()
    dp.finish_gradient_sync()
    try:
        opt.step()
    except RuntimeError as e:
        return str(e)
    return "no error"


def test_sharded_refuses_an_optimizer_that_cannot_update_by_shards():
    """A sharded DataParallel holds reduced values only in this rank's shard of flat.grad and
    relies on the optimizer to start the weight all-gathers: an optimizer whose param groups
    do not map onto the one flat buffer must raise, not fall back to a full-replica update
    (which would silently diverge the replicas)."""
    res = FakeWorld(2).run(_two_groups)
    for r in res:
        assert "shard_optimizer=True" in r and "param group" in r, res
