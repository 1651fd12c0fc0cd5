"""JSONL metrics logging (SURVEY §5 observability): one line per event per rank,
plus samples/sec and step-time reporting.  Replaces the reference's print/tqdm
bookkeeping (BAR/trainer.py:109-110,174) with machine-readable records."""
from __future__ import annotations

import json
import os
import time


class MetricsLogger:
    def __init__(self, path: str | None, rank: int = 0, also_print: bool = False):
        self.rank = rank
        self.also_print = also_print
        self.f = None
        if path:
            d = os.path.dirname(path)
            if d:
                os.makedirs(d, exist_ok=True)
            root, ext = os.path.splitext(path)
            self.path = f"{root}.rank{rank}{ext or '.jsonl'}"
            self.f = open(self.path, "a", buffering=1)
        self.t0 = time.time()

    def log(self, **rec):
        rec = {"t": round(time.time() - self.t0, 4), "rank": self.rank, **rec}
        line = json.dumps(rec, default=float)
        if self.f:
            self.f.write(line + "\n")
        if self.also_print:
            print(line, flush=True)

    def close(self):
        if self.f:
            self.f.close()
            self.f = None


def read_jsonl(path: str) -> list[dict]:
    with open(path) as f:
        return [json.loads(l) for l in f if l.strip()]
