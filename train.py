"""Training entry point (the reference's main.py): see ldnn/cli.py for the flags.

    python train.py --model enhanced_cnn --epochs_global 20 --epochs_local 5
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 train.py --sync_every step
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import ldnn.cli  # noqa: E402

if __name__ == "__main__":
    ldnn.cli.main()
