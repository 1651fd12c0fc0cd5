"""Graph-captured data-parallel steps (train/graphed.py GraphedDPStep): the backward is
a chain of graphs cut at the bucket-ready points with each bucket's collective issued
between two links of the chain (segmented), or one backward graph followed by every
collective (after); then the optimizer graph."""
import os
import socket
import subprocess
import sys

import pytest
import torch

import ldnn
from ldnn.models import CrossEntropyLoss, build_model, xavier_init
from ldnn.optim import SGD
from ldnn.parallel.comm import LocalComm
from ldnn.parallel.ddp import DataParallel
from ldnn.train.graphed import GraphedDPStep, GraphedStep

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _models(name, n):
    torch.manual_seed(0)
    ms = [build_model(name) for _ in range(n)]
    xavier_init(ms[0])
    for m in ms[1:]:
        m.load_state_dict(ms[0].state_dict())
    for m in ms:
        ldnn.prepare(m, "cuda")
    return ms


def _close_updates(pa, pb, p0, rel=2e-2):
    for a, b, r in zip(pa, pb, p0):
        da, db = (a.detach() - r).double(), (b.detach() - r).double()
        assert (da - db).norm().item() <= rel * db.norm().item() + 1e-6, ((da - db).norm().item(), db.norm().item())


@pytest.mark.parametrize("mode", ["segmented", "after"])
@pytest.mark.parametrize("comm_dtype", [None, torch.bfloat16])
def test_side_stream_collective_waits_for_its_bucket(comm_dtype, mode):
    """Ordering check without a second rank: the 'collective' doubles each bucket where
    the all-reduce would run (between two graphs of the chain for segmented).  Only if
    it runs after the bucket's gradients were written and before the optimizer is the
    result == plain SGD at twice the lr."""
    shape = (512, 1, 28, 28)
    m1, m2 = _models("lenet5", 2)
    crit = CrossEntropyLoss()
    dp = DataParallel(m1, LocalComm(), bucket_cap_mb=0.05, broadcast_init=False, comm_dtype=comm_dtype)
    assert len(dp.bucketer.buckets) >= 3
    o1, o2 = SGD(m1.parameters(), lr=0.01, momentum=0.0), SGD(m2.parameters(), lr=0.02, momentum=0.0)
    g = torch.Generator(device="cuda").manual_seed(1)
    xs = [torch.randn(*shape, device="cuda", generator=g).bfloat16() for _ in range(4)]
    ys = [torch.randint(0, 10, (shape[0],), device="cuda", generator=g) for _ in range(4)]
    p0 = [p.detach().clone() for p in m2.parameters()]
    # one eager step each first (optimizer state exists before capture), the same x2 on m1
    for m, o, k in ((m1, o1, 2.0), (m2, o2, 1.0)):
        o.zero_grad()
        crit(m(xs[0]), ys[0]).backward()
        m._ldnn_flat.grad.mul_(k)
        o.step()
    gd = GraphedDPStep(dp, crit, o1, xs[0], ys[0], mode=mode, comm_fn=lambda i, buf: buf.mul_(2.0))
    if mode == "segmented":   # one cut per bucket (+ the trailing piece of the backward)
        assert gd.n_segments >= len(dp.bucketer.buckets)
        assert sorted(i for iss in gd.issue for i in iss) == list(range(len(dp.bucketer.buckets)))
    gs = GraphedStep(m2, crit, o2, xs[0], ys[0], warmup=0)
    for i in range(1, 4):
        gd(xs[i], ys[i])
        gs(xs[i], ys[i])
    torch.cuda.synchronize()
    _close_updates(list(m1.parameters()), list(m2.parameters()), p0, rel=2e-2 if comm_dtype is None else 5e-2)


def test_rccl_world1_overlap_path(tmp_path):
    """The real RCCL path (TorchComm on a 1-rank communicator: the bucket all-reduces
    issued between the links of the backward chain) trains like the single-process
    graphed step, and records the same collective schedule as the eager fallback."""
    import torch.distributed as dist

    from ldnn.parallel.comm import TorchComm

    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        shape = (256, 1, 28, 28)
        m1, m2 = _models("lenet5", 2)
        crit = CrossEntropyLoss()
        comm = TorchComm()
        assert comm.device_collectives
        dp = DataParallel(m1, comm, bucket_cap_mb=0.05, broadcast_init=False)
        o1, o2 = SGD(m1.parameters(), lr=0.02, momentum=0.9), SGD(m2.parameters(), lr=0.02, momentum=0.9)
        g = torch.Generator(device="cuda").manual_seed(2)
        xs = [torch.randn(*shape, device="cuda", generator=g).bfloat16() for _ in range(5)]
        ys = [torch.randint(0, 10, (shape[0],), device="cuda", generator=g) for _ in range(5)]
        p0 = [p.detach().clone() for p in m2.parameters()]
        for m, o in ((m1, o1), (m2, o2)):
            o.zero_grad()
            crit(m(xs[0]), ys[0]).backward()
            o.step()
        gd = GraphedDPStep(dp, crit, o1, xs[0], ys[0])
        assert gd.mode == "segmented"
        gs = GraphedStep(m2, crit, o2, xs[0], ys[0], warmup=0)
        n0 = comm.schedule_digest()[0]
        gd(xs[1], ys[1])
        gs(xs[1], ys[1])
        n_graphed = comm.schedule_digest()[0] - n0
        assert n_graphed == len(dp.bucketer.buckets)
        for i in range(2, 5):
            gd(xs[i], ys[i])
            gs(xs[i], ys[i])
        # the odd-shaped last batch of an epoch falls back to the eager bucketed step
        gd(xs[0][:100], ys[0][:100])
        gs(xs[0][:100], ys[0][:100])
        torch.cuda.synchronize()
        _close_updates(list(m1.parameters()), list(m2.parameters()), p0)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("extra", [[], ["--shard"], ["--shard", "--optimizer", "adam"],
                                   ["--shard", "--comm-dtype", "bf16"], ["--gossip", "1"],
                                   ["--gossip", "2", "--optimizer", "adam"], ["--gossip", "1", "--comm-dtype", "bf16"]])
def test_graphed_dp_two_ranks_gloo_equals_big_batch(extra):
    """2 ranks (gloo, sharing the GPU) through train_local_epoch(graphs=True, dp=...)
    end with the parameters of ONE graphed rank on the concatenated batches -- also
    with the sharded step (reduce-scatter + sharded SGD / Adam + weight all-gather)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(ROOT, "scripts", "check_graphed_dp.py")] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "GRAPHED_DP_OK" in r.stdout, r.stdout[-3000:]


def test_segmented_weighted_allreduce_world1_identity():
    """--aggregation_type weighted on a world of one keeps the own gradient (Q4)."""
    shape = (128, 1, 28, 28)
    m1, m2 = _models("lenet5", 2)
    crit = CrossEntropyLoss()
    dp = DataParallel(m1, LocalComm(), bucket_cap_mb=0.05, broadcast_init=False, local_weight=0.8)
    assert not dp.bucketer.weighted
    o1, o2 = SGD(m1.parameters(), lr=0.02, momentum=0.9), SGD(m2.parameters(), lr=0.02, momentum=0.9)
    g = torch.Generator(device="cuda").manual_seed(3)
    xs = [torch.randn(*shape, device="cuda", generator=g).bfloat16() for _ in range(3)]
    ys = [torch.randint(0, 10, (shape[0],), device="cuda", generator=g) for _ in range(3)]
    p0 = [p.detach().clone() for p in m2.parameters()]
    for m, o in ((m1, o1), (m2, o2)):
        o.zero_grad()
        crit(m(xs[0]), ys[0]).backward()
        o.step()
    gd = GraphedDPStep(dp, crit, o1, xs[0], ys[0], mode="segmented", comm_fn=lambda i, buf: None)
    gs = GraphedStep(m2, crit, o2, xs[0], ys[0], warmup=0)
    for i in range(1, 3):
        gd(xs[i], ys[i])
        gs(xs[i], ys[i])
    torch.cuda.synchronize()
    _close_updates(list(m1.parameters()), list(m2.parameters()), p0)


def test_segmented_comm_stream_standin_overlaps():
    """A bandwidth-bound stand-in for each bucket's collective on its own HIP stream
    (parallel/overlap_probe.py) runs beside the remaining backward graphs: the step
    with the stand-in costs less than the step without it plus the stand-in's
    standalone time (no overlap at all would make them equal)."""
    from ldnn.parallel.overlap_probe import measure_overlap

    # (a timing claim: in the full suite a measurement has once landed while the GPU was still
    # busy with an earlier test's work -- every time 3-4x slower, the stand-in alone too -- so
    # it is taken up to three times and judged on the best one)
    runs = []
    for _ in range(3):
        r = measure_overlap("lenet5", batch=1024, bucket_mb=0.05, reps=64, steps=20, blocks=8)
        assert r["segments"] >= 3
        runs.append(r)
        if r["with_standin_ms"] < r["single_ms"] + r["standin_alone_ms"]:
            break
    assert any(r["with_standin_ms"] < r["single_ms"] + r["standin_alone_ms"] for r in runs), runs


def test_eager_fallback_and_replay_record_the_same_schedule():
    """A rank whose last batch is short runs the eager bucketed step while its peers
    replay the graph chain: both must record the same collectives, or
    Comm.check_schedule raises a false RankDivergenceError.  A 2-rank stand-in comm
    (identity collectives) keeps the bookkeeping of a real world > 1."""
    import hashlib

    class TwoRankEcho(LocalComm):
        world_size = 2

    shape = (128, 1, 28, 28)
    m1, = _models("lenet5", 1)
    crit = CrossEntropyLoss()
    comms = [TwoRankEcho(), TwoRankEcho()]
    dp = DataParallel(m1, comms[0], bucket_cap_mb=0.05, broadcast_init=False)
    o1 = SGD(m1.parameters(), lr=0.01, momentum=0.0)
    x = torch.randn(*shape, device="cuda").bfloat16()
    y = torch.randint(0, 10, (shape[0],), device="cuda")
    o1.zero_grad()
    crit(dp(x), y).backward()
    dp.finish_gradient_sync()
    o1.step()
    gd = GraphedDPStep(dp, crit, o1, x, y)
    digests = []
    for c, xb, yb in ((comms[0], x, y), (comms[1], x[:50], y[:50])):
        dp.comm = dp.bucketer.comm = gd.comm = c
        c._sched, c._nops = hashlib.sha1(), 0
        gd(xb, yb)    # full batch: graph chain; short batch: eager fallback
        digests.append(c.schedule_digest())
    torch.cuda.synchronize()
    assert digests[0] == digests[1] and digests[0][0] == len(dp.bucketer.buckets), digests


@pytest.mark.parametrize("name", ["resnet18", "enhanced_cnn"])
def test_fused_launches_fire_every_module_pre_hook(name):
    """conv2d_pair (a downsampling block's 3x3 + 1x1 shortcut in one launch) and gap_linear (pool +
    fc) stand in for several module calls: each module's forward pre-hook must still fire -- the
    sharded DP step cuts its graph chain there and waits for that bucket's weight all-gather
    (the shortcut's weights sat in bucket 0 of ResNet-18 and were read unwaited)."""
    (m,) = _models(name, 1)
    calls = {}

    def sharded(mod):   # (the sharded buckets hold the >= 2-D weights; 1-D ones are read from the
        # replicated fp32 master tail, which no all-gather writes)
        return any(p.dim() >= 2 for p in mod.parameters(recurse=False))

    for mod in m.modules():
        if sharded(mod):
            mod.register_forward_pre_hook(lambda mod, args: calls.__setitem__(id(mod), calls.get(id(mod), 0) + 1))
    shape = (8, 3, 224, 224) if name == "resnet18" else (8, 3, 32, 32)
    x = torch.randn(*shape, device="cuda").bfloat16()
    with torch.no_grad():
        m(x)
    owners = [mod for mod in m.modules() if sharded(mod)]
    missed = [type(mod).__name__ for mod in owners if calls.get(id(mod), 0) != 1]
    assert not missed, missed


def test_sharded_chain_waits_for_every_sharded_bucket_before_the_optimizer_reads():
    """With the shard layout of a world-8 stand-in, every sharded bucket holding a weight the
    forward reads is waited for by some forward link of GraphedDPStep (the first reader's hook)."""
    from ldnn.parallel.overlap_probe import ShardProbeComm

    (m,) = _models("resnet18", 1)
    comm = ShardProbeComm(torch.device("cuda"), world=8, reps=1, blocks=4)
    dp = DataParallel(m, comm, bucket_cap_mb=32.0, broadcast_init=False, shard_optimizer=True)
    opt = SGD(m.parameters(), lr=0.01, momentum=0.9)
    crit = CrossEntropyLoss()
    x = torch.randn(8, 3, 224, 224, device="cuda").bfloat16()
    y = torch.randint(0, 1000, (8,), device="cuda")
    opt.zero_grad()
    crit(dp(x), y).backward()
    dp.finish_gradient_sync()
    opt.step()
    dp.wait_gathers()
    gd = GraphedDPStep(dp, crit, opt, x, y)
    waited = {b for w in gd.waits for b in w}
    sharded = {i for i, b in enumerate(dp.bucketer.buckets) if b["sharded"]}
    assert sharded and sharded <= waited, (sharded, waited)
    # the first link that reads the shortcut conv's weights waits for their bucket: the
    # downsampling blocks' 1x1 convs are read by the paired launch, after their hooks fired
    gd(x, y)
    torch.cuda.synchronize()
