"""Checkpoint / resume equivalence and the CLI flag surface (SURVEY §4 'checkpoint', §5 config)."""
import os
import sys

import torch

import ldnn
from ldnn.cli import build_parser
from ldnn.models import CrossEntropyLoss
from ldnn.models.mlp import mlp2
from ldnn.optim import Adam, StepLR
from ldnn.utils.checkpoint import Checkpointer, load_checkpoint


def _step(m, opt, x, y):
    opt.zero_grad()
    loss = CrossEntropyLoss()(m(x), y)
    loss.backward()
    opt.step()
    return loss.item()


def test_save_load_gives_identical_next_step(tmp_path):
    torch.manual_seed(0)
    x, y = torch.randn(16, 784), torch.randint(0, 10, (16,))
    m = mlp2(784, 32, 10)
    ldnn.prepare(m, "cpu")
    opt = Adam(m.parameters(), lr=1e-2)
    sch = StepLR(opt, 1, gamma=0.5)
    for _ in range(3):
        _step(m, opt, x, y)
        sch.step()
    ck = Checkpointer(str(tmp_path), rank=0)
    p = ck.save(3, m, opt, sch, histories={"global_train_losses": [1.0, 0.5]}, extra={"note": "x"})
    ref_next = _step(m, opt, x, y)

    torch.manual_seed(99)
    m2 = mlp2(784, 32, 10)
    ldnn.prepare(m2, "cpu")
    opt2 = Adam(m2.parameters(), lr=1e-2)
    sch2 = StepLR(opt2, 1, gamma=0.5)
    sd = load_checkpoint(p, m2, opt2, sch2)
    assert sd["global_epoch"] == 3 and sd["histories"]["global_train_losses"] == [1.0, 0.5]
    assert opt2.param_groups[0]["lr"] == opt.param_groups[0]["lr"] and sch2.last_epoch == sch.last_epoch
    got_next = _step(m2, opt2, x, y)
    assert abs(got_next - ref_next) < 1e-6
    # reference state_dict key names survive the round trip
    assert set(torch.load(p, weights_only=True)["model"].keys()) == set(m.state_dict().keys())
    assert ck.latest() == p


def test_cli_accepts_every_reference_flag():
    args = build_parser().parse_args([
        "--local-rank", "0", "--backend", "gloo", "--epochs_local", "5", "--epochs_global", "20", "--batch_size", "64",
        "--lr", "0.001", "--time_limit", "60", "--prev_fraction", "0.5", "--next_fraction", "0.5",
        "--aggregation_type", "weighted", "--aggregation_by", "weights", "--local_weight", "0.5",
        "--fixed_ratio", "0.5", "--gpu_weight", "10", "--dist-url", "tcp://x",
    ])
    assert args.epochs_local == 5 and args.aggregation_type == "weighted" and args.fixed_ratio == 0.5
    # defaults match the reference (BAR/main.py:86-95)
    d = build_parser().parse_args([])
    assert (d.epochs_local, d.epochs_global, d.batch_size, d.lr, d.time_limit) == (5, 20, 64, 1e-3, 60)
    assert (d.aggregation_type, d.aggregation_by, d.local_weight) == ("equal", "gradients", 0.5)
    assert d.optimizer == "adam" and d.step_size == 25 and d.model == "enhanced_cnn"


def test_cli_single_process_cpu_run(tmp_path):
    from ldnn.cli import main

    res = main(["--model", "mlp2", "--dataset", "mnist", "--n_train", "800", "--n_test", "160", "--epochs_global",
                "2", "--epochs_local", "1", "--device", "cpu", "--quiet", "--out_dir", str(tmp_path), "--plots",
                str(tmp_path / "G"), "--checkpoint_every", "1"])
    assert len(res["histories"]) == 12 and "f1_macro" in res
    assert len(list((tmp_path / "G").glob("*.png"))) == 6
    # resume continues from the last checkpoint
    res2 = main(["--model", "mlp2", "--dataset", "mnist", "--n_train", "800", "--n_test", "160", "--epochs_global",
                 "3", "--epochs_local", "1", "--device", "cpu", "--quiet", "--out_dir", str(tmp_path), "--plots", "",
                 "--resume", "latest"])
    assert len(res2["histories"][4]) == 3  # 2 restored + 1 new global epoch


def test_cli_trace_phase_times(tmp_path):
    """--trace: roctx ranges (no-op without the native extension) + per-phase timers in metrics.jsonl."""
    import json

    from ldnn.cli import main
    from ldnn.utils import tracing

    try:
        main(["--model", "mlp2", "--dataset", "mnist", "--n_train", "400", "--n_test", "80", "--epochs_global",
              "1", "--epochs_local", "1", "--device", "cpu", "--quiet", "--out_dir", str(tmp_path), "--plots", "",
              "--no_eval", "--trace"])
    finally:
        tracing.enable(False)
    recs = [json.loads(l) for l in open(tmp_path / "metrics.rank0.jsonl")]
    ph = [r for r in recs if r.get("kind") == "phase_times"][0]["phases"]
    assert {"forward", "backward", "optimizer", "validate", "aggregate"} <= set(ph)
    n = ph["forward"]["count"]
    assert n > 0 and ph["backward"]["count"] == n and ph["optimizer"]["count"] == n


def test_phase_timer_disabled_is_free():
    from ldnn.utils.tracing import PhaseTimer

    t = PhaseTimer(enabled=False)
    with t.phase("x"):
        pass
    assert t.summary() == {}


def test_replace_follows_reference_variant():
    """--replace auto: with replacement for the class-skewed variants (DAR/DR/DDR
    dataloader.py:123,129) and the balanced double ring (BDR:94,100), without for BAR/BR."""
    p = build_parser()
    assert p.parse_args([]).replace == "auto" and p.parse_args(["--replace"]).replace == "on"
    assert p.parse_args(["--replace", "off"]).replace == "off"
    from ldnn.cli import resolve_replace

    assert resolve_replace("auto", None, "allreduce") is False
    assert resolve_replace("auto", None, "ring") is False
    assert resolve_replace("auto", None, "double_ring") is True
    assert resolve_replace("auto", 0.5, "allreduce") is True
    assert resolve_replace("off", 0.5, "ring") is False and resolve_replace("on", None, "ring") is True


def test_rank_without_its_extra_drops_rank0_shard(tmp_path):
    """A rank > 0 resuming a rank-0 checkpoint whose per-rank extra file is missing must
    not silently take rank 0's shard indices / partition RNG."""
    import numpy as np
    import pytest

    m = mlp2(784, 32, 10)
    ldnn.prepare(m, "cpu")
    opt = Adam(m.parameters(), lr=1e-2)
    p = Checkpointer(str(tmp_path), rank=0).save(2, m, opt, None, histories={},
                                                 extra={"indices_train": np.arange(5), "indices_val": np.arange(3),
                                                        "rng_state": {"a": 1}, "fixed_classes": [0, 1]})
    with pytest.warns(UserWarning, match="re-partitioned"):
        sd = load_checkpoint(p, m, opt, rank=1)
    assert "indices_train" not in sd["extra"] and "rng_state" not in sd["extra"]
    assert list(sd["extra"]["fixed_classes"]) == [0, 1]
    sd0 = load_checkpoint(p, m, opt, rank=0)
    assert "indices_train" in sd0["extra"]
