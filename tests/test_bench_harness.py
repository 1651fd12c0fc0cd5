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


def _configs_worker(rank, world, port, q):
    import importlib.util
    import types

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import datetime

    # (a short timeout: the healthy rank waits inside the failed config's collective until then)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=5))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    ctx = types.SimpleNamespace(world_size=world, rank=rank, backend="gloo", device="cpu")
    ran = []

    def run_fn(ctx, name, b, st, o):
        ran.append(name)
        if name == "bad" and rank == 1:
            raise RuntimeError("out of memory on rank 1 only")
        if name == "dead" and rank == 0:
            raise RuntimeError("HIP error: an illegal memory access was encountered")
        dist.all_reduce(__import__("torch").ones(1))   # a config's own collectives
        return {"ok": name}

    out = bench.run_configs(ctx, (("a", 1, 1, "sgd"), ("bad", 1, 1, "sgd"), ("c", 1, 1, "sgd")), run_fn)
    q.put((rank, out, list(ran)))
    dist.destroy_process_group()


def test_config_failure_on_one_rank_is_agreed_and_does_not_hang():
    """A secondary config that raises on ONE rank only: the failure flag travels on a side group
    (never paired with the config's own collectives), every rank records the config as failed
    and all ranks stop the config loop together (a lone failing rank sat in a barrier
    while its peers entered the next config's collectives)."""
    import socket

    import torch.multiprocessing as mp

    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_configs_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict((r, (o, ran)) for r, o, ran in (q.get(timeout=120) for _ in ps))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in (0, 1):
        out, ran = res[r]
        assert ran == ["a", "bad"]   # both stop after the failed config (the group may be broken)
        assert out["a_b1"] == {"ok": "a"} and "skipped" in out["c_b1"]
        assert "error" in out["bad_b1"]
    assert "out of memory" in res[1][0]["bad_b1"]["error"]
    # rank 0 left the config's own collective at the timeout (its own error), never paired it
    # with rank 1's failure flag
    assert "error" in res[0][0]["bad_b1"]
