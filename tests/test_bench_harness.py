"""bench.py's N-GPU harness contract (CPU checks: nothing here touches a GPU)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=120, env=env)


def test_world_size_must_match_gpus():
    """Under a launcher that started a different number of ranks than --gpus: a clean
    non-zero exit naming both numbers (no silent 1-rank run labelled n_gpus N)."""
    r = _run(["--gpus", "2"], {"RANK": "0", "WORLD_SIZE": "3", "LOCAL_RANK": "0"})
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "--gpus 2 but the launcher started 3 ranks" in r.stderr


def test_rccl_needs_one_gpu_per_rank():
    """--gpus N with RCCL on a node with fewer GPUs fails fast before spawning ranks
    (RCCL refuses two ranks on one GPU: profiles/rccl_two_ranks_one_gpu_r2.txt)."""
    import torch

    n = torch.cuda.device_count() + 1
    r = _run(["--gpus", str(n)])
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "needs" in r.stderr and "GPU" in r.stderr
