"""python scripts/overlap_probe.py --model resnet18 --batch 64 [--reps 4] -> one JSON line
(see ldnn/parallel/overlap_probe.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ldnn  # noqa: E402,F401
from ldnn.parallel.overlap_probe import main  # noqa: E402

if __name__ == "__main__":
    main()
