"""Run bench.py's secondary CNN configs alone (in the order given), with bench.py's own
construction and timing -- to separate a config's time from what ran before it in bench.py.
Usage: python scripts/bench_cfg.py enhanced_cnn:64:30:adam resnet18:256:8:sgd ..."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from ldnn.utils import distributed as D  # noqa: E402


def main():
    ctx = D.setup(None)
    for spec in sys.argv[1:]:
        name, b, st, o = spec.split(":")
        rec = bench.run_cnn(ctx, name, int(b), int(st), o)
        print(json.dumps({"spec": spec, "ms_per_step": rec["ms_per_step"]}), flush=True)


if __name__ == "__main__":
    main()
