"""Checkpoint / resume (the reference has none).

Format: one ``torch.save`` dict per file, loadable with ``weights_only=True``
(plain tensors, numbers, strings, lists, dicts, numpy arrays converted to tensors):

  model        state_dict with the reference's key names (prep.0.weight,
               layer1.0.conv1.weight, layer4.1.bn2.running_var, fc.bias, ...)
  optimizer    optimizer state_dict (fused flat buffers included)
  scheduler    LR scheduler state_dict
  global_epoch completed global epochs
  histories    the 12 metric histories (resume continues the curves)
  extra        shard indices, fixed classes, RNG state, config
  torch_rng    CPU / GPU RNG states

Synchronous modes (all replicas identical) are written by rank 0 only, plus a
small per-rank ``xtra_geNNNN_rankR.pt`` with each other rank's own shard indices
and partition-RNG state (so a resumed run re-partitions exactly as an
uninterrupted one); gossip / independent-worker modes (replicas differ) write one
full file per rank.  Writes go to a temp file then os.replace (atomic).
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch


def _to_safe(x):
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(x))
    if isinstance(x, dict):
        return {str(k): _to_safe(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_to_safe(v) for v in x]
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (np.floating,)):
        return float(x)
    return x


class Checkpointer:
    def __init__(self, directory: str, rank: int = 0, per_rank: bool = False, every: int = 1, keep: int = 2):
        self.dir = directory
        self.rank = rank
        self.per_rank = per_rank
        self.every = max(1, every)
        self.keep = keep
        os.makedirs(directory, exist_ok=True)

    def path(self, global_epoch: int, rank: int | None = None) -> str:
        r = self.rank if rank is None else rank
        suffix = f"_rank{r}" if self.per_rank else ""
        return os.path.join(self.dir, f"ckpt_ge{global_epoch:04d}{suffix}.pt")

    def latest(self) -> str | None:
        suffix = f"_rank{self.rank}.pt" if self.per_rank else ".pt"
        cands = sorted(f for f in os.listdir(self.dir) if f.startswith("ckpt_ge") and f.endswith(suffix)
                       and (self.per_rank or "_rank" not in f))
        return os.path.join(self.dir, cands[-1]) if cands else None

    def extra_path(self, global_epoch: int, rank: int | None = None) -> str:
        r = self.rank if rank is None else rank
        return os.path.join(self.dir, f"xtra_ge{global_epoch:04d}_rank{r}.pt")

    def save(self, global_epoch, model, optimizer=None, scheduler=None, histories=None, extra=None, config=None):
        if global_epoch % self.every:
            return None
        if not self.per_rank and self.rank != 0:
            p = self.extra_path(global_epoch)
            torch.save({"format": "ldnn-xtra-v1", "global_epoch": int(global_epoch), "extra": _to_safe(extra or {})},
                       p + ".tmp")
            os.replace(p + ".tmp", p)
            self._prune()
            return p
        sd = {
            "format": "ldnn-ckpt-v1",
            "global_epoch": int(global_epoch),
            "model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
            "optimizer": _to_safe(optimizer.state_dict()) if optimizer is not None else None,
            "scheduler": scheduler.state_dict() if scheduler is not None else None,
            "histories": histories,
            "extra": _to_safe(extra or {}),
            "config": json.dumps(config or {}),
            "torch_rng": torch.get_rng_state(),
        }
        if torch.cuda.is_available():
            sd["cuda_rng"] = torch.cuda.get_rng_state()
        p = self.path(global_epoch)
        tmp = p + ".tmp"
        torch.save(sd, tmp)
        os.replace(tmp, p)
        self._prune()
        return p

    def _prune(self):
        if not self.per_rank and self.rank != 0:
            files = sorted(f for f in os.listdir(self.dir) if f.startswith("xtra_ge") and
                           f.endswith(f"_rank{self.rank}.pt"))
        else:
            suffix = f"_rank{self.rank}.pt" if self.per_rank else ".pt"
            files = sorted(f for f in os.listdir(self.dir) if f.startswith("ckpt_ge") and f.endswith(suffix)
                           and (self.per_rank or "_rank" not in f))
        for f in files[: max(0, len(files) - self.keep)]:
            try:
                os.remove(os.path.join(self.dir, f))
            except OSError:
                pass


def load_checkpoint(path: str, model, optimizer=None, scheduler=None, map_location="cpu",
                    rank: int | None = None) -> dict:
    """Restore model / optimizer / scheduler (and the torch CPU / GPU RNG) in place;
    returns the checkpoint dict.  For a rank-0 (synchronous-mode) checkpoint,
    ``rank`` > 0 swaps in that rank's own ``extra`` (shards, partition RNG)."""
    sd = torch.load(path, map_location=map_location, weights_only=True)
    base = os.path.basename(path)
    if rank and "_rank" not in base and base.startswith("ckpt_ge"):
        xp = os.path.join(os.path.dirname(path), f"xtra_ge{int(sd['global_epoch']):04d}_rank{rank}.pt")
        if os.path.exists(xp):
            sd["extra"] = torch.load(xp, map_location=map_location, weights_only=True)["extra"]
        else:
            # rank 0's shard indices / partition RNG are NOT this rank's: drop them (the
            # caller re-partitions from its own seed) instead of resuming every rank on
            # rank 0's shard with rank 0's draws (e.g. a non-shared filesystem, or a
            # checkpoint written before per-rank extras existed)
            import warnings

            warnings.warn(f"{xp} not found: rank {rank} resumes without its saved shard / partition RNG "
                          "(re-partitioned from the seed)")
            ex = dict(sd.get("extra") or {})
            for k in ("indices_train", "indices_val", "rng_state"):
                ex.pop(k, None)
            sd["extra"] = ex
    with torch.no_grad():
        model.load_state_dict(sd["model"])
    for m in model.modules():
        f = getattr(m, "_ldnn_flat", None)
        if f is not None:
            f.refresh_shadow()
            break
    if optimizer is not None and sd.get("optimizer") is not None:
        optimizer.load_state_dict(sd["optimizer"])
    if scheduler is not None and sd.get("scheduler") is not None:
        scheduler.load_state_dict(sd["scheduler"])
    if "torch_rng" in sd:
        torch.set_rng_state(sd["torch_rng"])
    if "cuda_rng" in sd and torch.cuda.is_available():
        torch.cuda.set_rng_state(sd["cuda_rng"])
    return sd
