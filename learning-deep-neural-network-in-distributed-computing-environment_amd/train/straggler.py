"""Working straggler cutoff (SURVEY §0.1 Q5, §2.1 A29, §5 failure detection).

The reference's finish-signal / time-limit protocol never fires: the flag is
reset every global epoch and only raised after the local loop
(BAR/trainer.py:42,113-119,134-139).  Its intent -- once the first worker has
finished its local epochs, the others get `time_limit` seconds before they are
cut off -- is implemented here so that every rank issues exactly the same
sequence of collectives:

* training is divided into rounds of `check_every` optimizer steps;
* after each round every rank joins ONE small all-reduce of
  [finished?, deadline passed?];
* a rank that has finished keeps joining rounds (idle) until everybody is done
  or the deadline passes; the deadline clock starts, on every rank, at the same
  round -- the first one in which some rank reported "finished" -- so the
  decision to stop is collective and identical everywhere.
"""
from __future__ import annotations

import math
import time

import torch

from ..parallel.comm import SUM, Comm


class StopLocalTraining(Exception):
    pass


class StragglerCutoff:
    def __init__(self, comm: Comm, time_limit: float, check_every: int = 20, device="cpu"):
        self.comm = comm
        self.time_limit = float(time_limit)
        self.check_every = max(1, int(check_every))
        self.device = torch.device(device)
        self.enabled = comm.world_size > 1 and math.isfinite(self.time_limit) and self.time_limit >= 0
        self.reset()

    def reset(self):
        self.done = False
        self.stop = False
        self.t_first_done: float | None = None
        self.rounds = 0
        self.cut = False  # this rank was cut short

    def _round(self) -> bool:
        over = self.t_first_done is not None and (time.perf_counter() - self.t_first_done) > self.time_limit
        t = torch.tensor([1.0 if self.done else 0.0, 1.0 if over else 0.0], device=self.device)
        self.comm.all_reduce(t, SUM)
        n_done, n_over = t.tolist()
        self.rounds += 1
        if n_done > 0 and self.t_first_done is None:
            self.t_first_done = time.perf_counter()
        if n_done >= self.comm.world_size or n_over > 0:
            self.stop = True
        return self.stop

    def step(self, step_index: int):
        """Call after every optimizer step; raises StopLocalTraining on a collective cutoff."""
        if not self.enabled or (step_index + 1) % self.check_every:
            return
        if self._round():
            self.cut = True
            raise StopLocalTraining()

    def finish(self):
        """This rank finished its local epochs: keep joining rounds until the collective stop."""
        if not self.enabled:
            return
        self.done = True
        while not self.stop:
            self._round()
