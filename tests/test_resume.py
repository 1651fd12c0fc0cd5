"""Faithful resume (SURVEY §5 checkpoint/resume; BAR/trainer.py:179-188 re-partitions
every global epoch from an RNG): 2 gloo ranks on the CPU train 3 global epochs
uninterrupted, vs 1 epoch -> checkpoint -> a FRESH pair of processes resuming for 2
more.  The 12 histories and every rank's final parameters must be bit-identical, in
the reference schedule (per-rank checkpoints) and with per-step all-reduce (rank-0
checkpoint + per-rank shard / RNG extras)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(out, epochs, extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(_port()), os.path.join(ROOT, "train.py"), "--model", "mlp2", "--dataset", "mnist",
           "--n_train", "1500", "--n_test", "100", "--epochs_global", str(epochs), "--epochs_local", "2",
           "--device", "cpu", "--quiet", "--out_dir", out, "--plots", "", "--checkpoint_every", "1",
           "--partition_rule", "equal", "--time_limit", "0", "--lr", "0.01", "--seed", "3", "--no_eval",
           "--batch_size", "32"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]


def _params(path):
    return torch.load(path, weights_only=True)["model"]


@pytest.mark.slow
@pytest.mark.parametrize("mode", ["reference", "step_allreduce"])
def test_resume_is_bit_identical(tmp_path, mode):
    extra = ["--aggregation_by", "weights", "--topology", "ring"] if mode == "reference" else \
        ["--sync_every", "step", "--partition", "skewed"]
    a, b = str(tmp_path / "a"), str(tmp_path / "b")
    _run(a, 3, extra)                          # uninterrupted
    _run(b, 1, extra)                          # 1 global epoch, checkpoint
    _run(b, 3, extra + ["--resume", "latest"])  # fresh processes: resume for 2 more
    # the second invocation really resumed: global epochs 1 | 2, 3 (not 1 | 1, 2, 3)
    for r in (0, 1):
        recs = [json.loads(l) for l in open(os.path.join(b, f"metrics.rank{r}.jsonl")) if l.strip()]
        assert [x["global_epoch"] for x in recs if x.get("kind") == "global_epoch"] == [1, 2, 3]
    ha = json.load(open(os.path.join(a, "histories.json")))["histories"]
    hb = json.load(open(os.path.join(b, "histories.json")))["histories"]
    assert ha == hb
    per_rank = mode == "reference"
    names = [f"ckpt_ge0003_rank{r}.pt" for r in (0, 1)] if per_rank else ["ckpt_ge0003.pt"]
    for n in names:
        pa, pb = _params(os.path.join(a, "ckpt", n)), _params(os.path.join(b, "ckpt", n))
        assert pa.keys() == pb.keys()
        for k in pa:
            assert torch.equal(pa[k], pb[k]), (n, k)
    if not per_rank:  # rank 1's shard + RNG travelled in its extra file
        xa = torch.load(os.path.join(a, "ckpt", "xtra_ge0003_rank1.pt"), weights_only=True)["extra"]
        xb = torch.load(os.path.join(b, "ckpt", "xtra_ge0003_rank1.pt"), weights_only=True)["extra"]
        assert torch.equal(xa["indices_train"], xb["indices_train"])
