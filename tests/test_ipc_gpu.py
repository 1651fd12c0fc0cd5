"""One-shot IPC all-reduce (parallel/ipc.py, csrc/kernels/ipc.hip) across processes:
two and three ranks sharing the box's GPU, fp32 / bf16 sums vs exact expectations
over many back-to-back calls (scripts/oneshot_check.py does the per-rank work)."""
import json
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("nproc,port", [(2, 29611), (3, 29612)])
def test_oneshot_all_reduce_multiprocess(nproc, port):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "scripts", "oneshot_check.py")]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    # ranks print concurrently: their JSON objects may share a line
    lines = [json.loads(m) for m in re.findall(r"\{[^{}]*\}", r.stdout)]
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert len(lines) == nproc and all(d["ok"] for d in lines), lines


@pytest.mark.parametrize("nproc", [2, 3])
def test_graphed_dp_with_oneshot_matches_plain_collectives(nproc):
    """the graphed DP training path (segmented GraphedDPStep + the eager
    fallback for the odd last batch) with every <= 4 MiB bucket on the one-shot IPC
    all-reduce ends with the parameters of the same run on the process group's
    all-reduce, and the one-shot kernel was actually used."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "scripts", "check_graphed_dp.py"), "--oneshot", "--steps", "4"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "GRAPHED_DP_OK" in r.stdout, r.stdout[-3000:]
    used = [int(m) for m in re.findall(r"one-shot calls (\d+)", r.stdout)]
    assert len(used) == nproc and all(u > 0 for u in used), r.stdout[-2000:]
