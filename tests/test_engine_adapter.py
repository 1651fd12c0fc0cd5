"""The static MLP engine behind the reference API (train/engine_adapter.py): train_global /
train_local_epoch / StepLR / checkpoint drive StaticMLPEngine (BAR/main.py:57-59, BAR/trainer.py:11,194)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

from ldnn.train import engine_adapter as EA


class FakeEngine:
    """CPU stand-in with the engine's step / stats contract: stats rows accumulate
    (loss sum, #correct) on the device; step() adds this batch's contribution."""

    def __init__(self, B):
        self.B, self.device, self.distributed = B, torch.device("cpu"), False
        self.stats = torch.zeros(3, 2)
        self.lr, self.steps, self.synced = None, 0, 0
        self.x = None

    def set_lr(self, lr):
        self.lr = lr

    def reset_stats(self):
        self.stats.zero_()

    def load_batch(self, x, y):
        self.x, self.y = x, y

    def step(self):
        self.steps += 1
        # loss of this batch = mean of x; split over the slots like the head kernel's per-workgroup sums
        self.stats[self.steps % 3, 0] += float(self.x.float().mean()) * self.B
        self.stats[0, 1] += float((self.y == 0).sum())

    def eager_step(self, x, y):   # the partial batch: same stats contract
        self.eager = getattr(self, "eager", 0) + 1
        self.stats[0, 0] += float(x.float().mean()) * y.numel()
        self.stats[0, 1] += float((y == 0).sum())

    def dp_tail_step(self, x=None, y=None):   # data-parallel tail step: any size, or none
        self.tails = getattr(self, "tails", []) + [0 if y is None else y.numel()]
        if y is not None:
            self.stats[0, 0] += float(x.float().mean()) * y.numel()
            self.stats[0, 1] += float((y == 0).sum())

    def sync(self):
        self.synced += 1

    def gather_master(self):
        pass


class _Model(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.fc = torch.nn.Linear(2, 2)


def _loader(B, n_full, tail):
    batches = [(torch.full((B, 2), float(i + 1)), torch.tensor([0] * (B // 2) + [1] * (B - B // 2)))
               for i in range(n_full)]
    if tail:
        batches.append((torch.full((tail, 2), 99.0), torch.zeros(tail, dtype=torch.long)))

    class L(list):
        num_samples = B * n_full + tail

    return L(batches)


@pytest.mark.filterwarnings(r"ignore:Detected call of `lr_scheduler.step\(\)`")
def test_engine_local_epoch_per_batch_losses_and_partial_batch_trained():
    """Every batch is trained, the trailing partial one too (BAR/trainer.py:202-216):
    it runs the engine's eager_step; per-batch losses are per-batch means."""
    B = 8
    m = EA.EngineModule(_Model(), FakeEngine(B))
    opt = torch.optim.SGD(m.module.parameters(), lr=0.25)
    sch = torch.optim.lr_scheduler.StepLR(opt, 1, gamma=0.5)
    loss, acc, bl = EA.engine_local_epoch(m, _loader(B, 4, 3), opt, sch)
    assert m.engine.lr == 0.25 and opt.param_groups[0]["lr"] == 0.125   # synced before, stepped after
    assert bl == pytest.approx([1.0, 2.0, 3.0, 4.0, 99.0]) and loss == pytest.approx(109.0 / 5)
    assert acc == pytest.approx(100.0 * (4 * 4 + 3) / (4 * B + 3))
    assert EA.engine_local_epoch.last_skipped == 0 and EA.engine_local_epoch.last_samples == 4 * B + 3
    assert m.engine.steps == 4 and m.engine.eager == 1
    # a data-parallel engine: the full steps, then ONE tail step on every rank (its partial
    # batch, a full batch past the common step count, or nothing) -- VERDICT r3 #7
    md = EA.EngineModule(_Model(), FakeEngine(B))
    md.engine.distributed = True
    _, _, bld = EA.engine_local_epoch(md, _loader(B, 4, 3), opt, None)
    assert bld == pytest.approx([1.0, 2.0, 3.0, 4.0, 99.0]) and EA.engine_local_epoch.last_skipped == 0
    assert md.engine.steps == 4 and md.engine.tails == [3]
    md2 = EA.EngineModule(_Model(), FakeEngine(B))   # shard ran out: a sample-less tail step
    md2.engine.distributed = True
    _, _, bld2 = EA.engine_local_epoch(md2, _loader(B, 4, 0), opt, None, max_steps=4)
    assert bld2 == pytest.approx([1.0, 2.0, 3.0, 4.0]) and md2.engine.tails == [0]
    md3 = EA.EngineModule(_Model(), FakeEngine(B))   # longer shard: step 3's full batch is the tail, 4 skipped
    md3.engine.distributed = True
    _, _, bld3 = EA.engine_local_epoch(md3, _loader(B, 4, 3), opt, None, max_steps=2)
    assert bld3 == pytest.approx([1.0, 2.0, 3.0]) and md3.engine.tails == [B]
    assert EA.engine_local_epoch.last_skipped == B + 3
    # max_steps caps the steps (per-step DP keeps ranks aligned)
    m2 = EA.EngineModule(_Model(), FakeEngine(B))
    _, _, bl2 = EA.engine_local_epoch(m2, _loader(B, 4, 0), opt, None, max_steps=2)
    assert bl2 == pytest.approx([1.0, 2.0]) and m2.engine.steps == 2
    assert m.full_batches(_loader(B, 4, 3)) == 4


def test_engine_module_keeps_model_keys():
    inner = _Model()
    m = EA.EngineModule(inner, FakeEngine(4))
    assert set(m.state_dict().keys()) == set(inner.state_dict().keys())
    assert "engine" not in dict(m.named_modules())


def test_resolve_engine_cpu():
    from ldnn.cli import build_parser, resolve_engine
    from ldnn.models.mlp import mlp2

    a = build_parser().parse_args(["--model", "mlp2"])
    assert resolve_engine(a, mlp2(), torch.device("cpu"), 1) is False
    a = build_parser().parse_args(["--model", "mlp2", "--engine", "static"])
    with pytest.raises(SystemExit):
        resolve_engine(a, mlp2(), torch.device("cpu"), 1)


# ------------------------------------------------------------------------ GPU
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _train(out, epochs, extra=(), nproc=2):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(nproc), "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "train.py"), "--model", "mlp3",
           "--dataset", "mnist", "--n_train", "2560", "--n_test", "256", "--batch_size", "128", "--epochs_global",
           str(epochs), "--epochs_local", "2", "--optimizer", "sgd", "--lr", "0.05", "--sync_every", "step",
           "--backend", "gloo", "--engine", "static", "--quiet", "--plots", "", "--out_dir", str(out),
           "--checkpoint_every", "1", "--partition_rule", "equal", "--time_limit", "0", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    with open(os.path.join(out, "histories.json")) as f:
        return json.load(f)


@pytest.mark.gpu
def test_cli_static_engine_gloo_two_ranks_resume(tmp_path):
    """train.py --engine static --sync_every step on 2 gloo ranks (one GPU): the 12
    histories, per-epoch samples/s in metrics.jsonl, and a checkpoint that resumes to
    the same trajectory as an uninterrupted run."""
    full = _train(tmp_path / "full", 3)
    h = full["histories"]
    assert len(h) == 12 and len(h[4]) == 3 and all(v == v for v in h[4])
    assert h[4][-1] < h[4][0]   # it learns
    recs = [json.loads(l) for l in open(tmp_path / "full" / "metrics.rank0.jsonl")]
    cfg = next(r for r in recs if r.get("kind") == "config")
    assert cfg["resolved_engine"] == "static"
    ge = [r for r in recs if r.get("kind") == "global_epoch"]
    assert len(ge) == 3 and all(r["samples"] > 0 and r["samples_per_s"] > 0 for r in ge)

    _train(tmp_path / "part", 2)
    res = _train(tmp_path / "part", 3, ("--resume", "latest"))
    r = res["histories"]
    assert len(r[4]) == 3
    torch.testing.assert_close(torch.tensor(r[4]), torch.tensor(h[4]), rtol=2e-3, atol=2e-3)
    torch.testing.assert_close(torch.tensor(r[6]), torch.tensor(h[6]), rtol=2e-3, atol=2e-3)
    a = torch.load(tmp_path / "full" / "ckpt" / "ckpt_ge0003.pt", weights_only=True)
    b = torch.load(tmp_path / "part" / "ckpt" / "ckpt_ge0003.pt", weights_only=True)
    for k in a["model"]:
        torch.testing.assert_close(a["model"][k], b["model"][k], rtol=2e-3, atol=2e-4)
    assert "ldnn_engine_state" in a["optimizer"] and a["optimizer"]["ldnn_engine_state"]["mom"] is not None


@pytest.mark.gpu
def test_static_engine_global_epoch_schedule_single_process(tmp_path):
    """Reference schedule (--sync_every global_epoch) with the engine as an independent
    replica: StepLR drives the engine's lr, evaluation runs on the engine's weights."""
    from ldnn.cli import main

    res = main(["--model", "mlp2", "--dataset", "mnist", "--n_train", "1600", "--n_test", "320", "--batch_size",
                "100", "--epochs_global", "2", "--epochs_local", "2", "--optimizer", "adam", "--lr", "1e-3",
                "--step_size", "1", "--engine", "static", "--quiet", "--plots", "", "--out_dir", str(tmp_path)])
    h = res["histories"]
    assert len(h) == 12 and len(h[9]) == 4 and res["test_acc"] > 50.0
