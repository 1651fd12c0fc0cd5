"""The graph-captured static MLP engine trains like a plain PyTorch fp32 model."""
import pytest
import torch

import ldnn
from ldnn.models.mlp import mlp3
from ldnn.train.static_mlp import OptimConfig, StaticMLPEngine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("library", [False, True])
@pytest.mark.parametrize("opt", ["sgd", "adam"])
@pytest.mark.parametrize("graphs", [False, True])
def test_engine_matches_fp32_reference(opt, graphs, library):
    torch.manual_seed(0)
    B = 256
    model = mlp3(784, 512, 10)
    ref = torch.nn.Sequential(torch.nn.Linear(784, 512), torch.nn.ReLU(), torch.nn.Linear(512, 512),
                              torch.nn.ReLU(), torch.nn.Linear(512, 10))
    for dst, src in zip(ref.parameters(), model.parameters()):
        dst.data.copy_(src.data)
    ref = ref.cuda()
    cfg = OptimConfig(opt, lr=0.05 if opt == "sgd" else 1e-3, momentum=0.9)
    eng = StaticMLPEngine(model, B, cfg, use_graphs=graphs, library_gemms=library)
    assert any(eng._lib_wgrad) == library and any(eng._lib_fwd) == library
    if opt == "sgd":
        ropt = torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9)
    else:
        ropt = torch.optim.Adam(ref.parameters(), lr=1e-3)
    g = torch.Generator(device="cuda").manual_seed(1)
    xs = [torch.randn(B, 784, device="cuda", generator=g) for _ in range(3)]
    ys = [torch.randint(0, 10, (B,), device="cuda", generator=g) for _ in range(3)]
    losses, rlosses = [], []
    for step in range(8):
        x, y = xs[step % 3], ys[step % 3]
        eng.reset_stats()
        eng.load_batch(x.bfloat16(), y)
        eng.step()
        losses.append(eng.read_stats(B)[0])
        ropt.zero_grad()
        out = ref(x.bfloat16().float())
        loss = torch.nn.functional.cross_entropy(out, y)
        loss.backward()
        ropt.step()
        rlosses.append(loss.item())
    for a, b in zip(losses, rlosses):
        assert abs(a - b) < 0.03 * max(1.0, abs(b)), (losses, rlosses)
    # parameters stayed close to the fp32 reference
    for p, q in zip(model.parameters(), ref.parameters()):
        assert (p.detach() - q.detach()).abs().max().item() < 2e-2


def test_graph_replay_matches_eager_with_splitk():
    """Graph-captured steps (incl. split-K zero-fill + atomics) == eager steps."""
    torch.manual_seed(0)
    B = 1024
    m1 = mlp3(784, 512, 10)
    m2 = mlp3(784, 512, 10)
    m2.load_state_dict(m1.state_dict())
    e1 = StaticMLPEngine(m1, B, OptimConfig("sgd", lr=0.05, momentum=0.9), use_graphs=True)
    e2 = StaticMLPEngine(m2, B, OptimConfig("sgd", lr=0.05, momentum=0.9), use_graphs=False)
    g = torch.Generator(device="cuda").manual_seed(3)
    for i in range(7):
        x = torch.randn(B, 784, device="cuda", generator=g).bfloat16()
        y = torch.randint(0, 10, (B,), device="cuda", generator=g)
        for e in (e1, e2):
            e.load_batch(x, y)
            e.step()
    torch.cuda.synchronize()
    # identical up to the arrival order of the split-K / bias-gradient fp32 atomics
    torch.testing.assert_close(e1.flat.master, e2.flat.master, rtol=1e-6, atol=1e-8)


@pytest.mark.parametrize("nproc,extra", [(2, []), (3, []), (2, ["--tail", "2,0"]), (3, ["--tail", "5,256,0"]),
                                         (2, ["--tail", "7,3", "--optimizer", "adam"]),
                                         (2, ["--tail", "7,3", "--shard", "0"]),
                                         # bf16 gradient reduce-scatter: 20 steps of the
                                         # headline's bucket layout (W2+W1 | W0+biases) within the same
                                         # 2e-2 x max|param| (+1e-3) of the fp32 single-rank reference
                                         (3, ["--comm-dtype", "bf16", "--steps", "20", "--hidden", "4096",
                                              "--cap", str(8 << 20)]),
                                         (2, ["--comm-dtype", "bf16", "--tail", "7,3"]),
                                         # Adam divides by sqrt(v): a near-zero gradient element whose bf16
                                         # sum flips sign moves by 2 lr, so the bound is looser (measured
                                         # 0.115 x max|param| after 7 steps + tail at lr 1e-3)
                                         (2, ["--comm-dtype", "bf16", "--tail", "7,3", "--optimizer", "adam",
                                              "--tol", "0.2"])])
def test_multirank_static_engine_gloo_two_ranks_one_gpu(nproc, extra):
    """The bucketed multi-rank step (sharded optimizer: reduce-scatter between graph
    segments, shard update, weight all-gather, fp32 bias refresh from the shard
    owners) equals one rank on the concatenated batch, and every rank's forward reads
    the same fp32 biases (2 / 3 ranks share the GPU via gloo).  ``--tail``: then one
    dp_tail_step with per-rank batches of any size (partial, full, none) == the single
    rank's eager_step on the concatenated tail (the DP engine trains the
    trailing partial batch)."""
    import os
    import socket
    import subprocess
    import sys

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(nproc), "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(root, "scripts", "check_static_dp.py"), "--backend", "gloo",
           "--hidden", "512", "--batch", "1024" if not extra else "256", "--steps", "7"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "BIASES_CONSISTENT" in r.stdout, r.stdout[-3000:]
    assert "STATIC_DP_OK" in r.stdout and "REPLICAS_IDENTICAL" in r.stdout, r.stdout[-3000:]


@pytest.mark.parametrize("opt,comm", [("sgd", None), ("adam", None), ("sgd", torch.bfloat16)])
def test_sharded_optimizer_path_on_rccl_single_rank(opt, comm, tmp_path):
    """The reduce-scatter / sharded-optimizer / in-place all-gather path on a real RCCL
    communicator (world 1, forced), graphs on, several buckets: identical to the
    single-segment engine.  comm bf16: the gradient buckets staged in bf16 (the 4096-wide
    layer's wgrad writes bf16 directly, the rest is cast) and reduce-scattered in bf16 --
    equal to the fp32 engine up to the gradients' bf16 rounding."""
    import torch.distributed as dist

    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        torch.manual_seed(0)
        B, H = (512, 1024) if comm is None else (512, 4096)
        m1, m2 = mlp3(784, H, 10), mlp3(784, H, 10)
        m2.load_state_dict(m1.state_dict())
        cfg = OptimConfig(opt, lr=0.05 if opt == "sgd" else 1e-3, momentum=0.9)
        e1 = StaticMLPEngine(m1, B, cfg, use_graphs=True, shard_optimizer=True,
                             bucket_cap_elems=(1 << 18) if comm is None else (8 << 20), comm_dtype=comm)
        e2 = StaticMLPEngine(m2, B, cfg, use_graphs=True)
        assert e1.shard and len(e1.buckets) >= 2
        if comm is not None:   # the 4096 x 4096 wgrad is a plain GEMM: its bf16 output goes straight to the stage
            assert e1.comm_bf16 and e1.dWb[1] is not None
        g = torch.Generator(device="cuda").manual_seed(4)
        for step in range(6):
            x = torch.randn(B, 784, device="cuda", generator=g).bfloat16()
            y = torch.randint(0, 10, (B,), device="cuda", generator=g)
            for e in (e1, e2):
                e.load_batch(x, y)
                e.step()
        e1.gather_master()
        torch.cuda.synchronize()
        for p, q in zip(m1.parameters(), m2.parameters()):
            if comm is None:
                torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-5, atol=1e-6)
            else:   # 6 SGD steps on bf16-rounded gradients
                torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-2, atol=2e-3 * q.abs().max().item())
        assert torch.equal(e1.flat.shadow, e1.flat.master.bfloat16())
    finally:
        dist.destroy_process_group()


def test_wgrad_inlaunch_splitk_combine_matches_unsplit():
    """A wgrad on the in-launch split-K combine path (1024 x 1024 layer: 64 tiles
    -> 4 slices) trains like the engine without it, and its steps are replayable
    from a graph."""
    torch.manual_seed(0)
    B = 2048
    m1, m2 = mlp3(784, 1024, 10), mlp3(784, 1024, 10)
    m2.load_state_dict(m1.state_dict())
    e1 = StaticMLPEngine(m1, B, OptimConfig("sgd", lr=0.05, momentum=0.9), use_graphs=True, library_gemms=False)
    e2 = StaticMLPEngine(m2, B, OptimConfig("sgd", lr=0.05, momentum=0.9), use_graphs=False, wgrad_combine=False,
                         library_gemms=False)
    assert any(w is not None for w in e1._wgrad_ws) and all(w is None for w in e2._wgrad_ws)
    g = torch.Generator(device="cuda").manual_seed(7)
    for i in range(6):
        x = torch.randn(B, 784, device="cuda", generator=g).bfloat16()
        y = torch.randint(0, 10, (B,), device="cuda", generator=g)
        for e in (e1, e2):
            e.load_batch(x, y)
            e.step()
    torch.cuda.synchronize()
    torch.testing.assert_close(e1.flat.master, e2.flat.master, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("B", [1024, 4096])
def test_library_gemm_engine_matches_native_engine(B):
    """hipBLASLt plain GEMMs (fp32 wgrads, bias+ReLU forwards,
    dgrads + the fused dReLU/bias-grad pass) inside the graph-captured step == the all-ldnn-kernel engine, up to
    bf16 rounding of the bias in the forward."""
    torch.manual_seed(0)
    m1, m2 = mlp3(784, 1024, 10), mlp3(784, 1024, 10)
    m2.load_state_dict(m1.state_dict())
    cfg = OptimConfig("sgd", lr=0.05, momentum=0.9)
    e1 = StaticMLPEngine(m1, B, cfg, use_graphs=True, library_gemms=True)
    e2 = StaticMLPEngine(m2, B, cfg, use_graphs=True, library_gemms=False)
    assert any(e1._lib_dgrad) and not any(e2._lib_dgrad)
    g = torch.Generator(device="cuda").manual_seed(5)
    l1, l2 = [], []
    for i in range(6):
        x = torch.randn(B, 784, device="cuda", generator=g).bfloat16()
        y = torch.randint(0, 10, (B,), device="cuda", generator=g)
        for e, ls in ((e1, l1), (e2, l2)):
            e.reset_stats()
            e.load_batch(x, y)
            e.step()
            ls.append(e.read_stats(B)[0])
    torch.cuda.synchronize()
    for a, b in zip(l1, l2):
        assert abs(a - b) < 1e-2 * max(1.0, abs(b)), (l1, l2)
    torch.testing.assert_close(e1.flat.master, e2.flat.master, rtol=2e-2, atol=2e-3)


def test_fused_head_dgrad_engine_matches_separate_dgrad():
    """fuse_head_dgrad=True (the head kernel writes dz_{L-1} and the previous bias
    gradient) trains exactly like the separate K = 16 dgrad GEMM path."""
    torch.manual_seed(0)
    B = 512
    m1, m2 = mlp3(784, 1024, 10), mlp3(784, 1024, 10)
    m2.load_state_dict(m1.state_dict())
    cfg = OptimConfig("sgd", lr=0.05, momentum=0.9)
    e1 = StaticMLPEngine(m1, B, cfg, use_graphs=True, fuse_head_dgrad=True)
    e2 = StaticMLPEngine(m2, B, cfg, use_graphs=True, fuse_head_dgrad=False)
    assert e1.head_dgrad and not e2.head_dgrad
    g = torch.Generator(device="cuda").manual_seed(6)
    for i in range(5):
        x = torch.randn(B, 784, device="cuda", generator=g).bfloat16()
        y = torch.randint(0, 10, (B,), device="cuda", generator=g)
        for e in (e1, e2):
            e.load_batch(x, y)
            e.step()
    torch.cuda.synchronize()
    torch.testing.assert_close(e1.flat.master, e2.flat.master, rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("act", ["relu", "sigmoid"])
def test_library_dgrad_matches_fused_dgrad(act):
    """hipBLASLt dgrad + fused act'/bias-grad pass (library_dgrad) == ldnn's dgrad with
    the activation derivative and bias column sums in its MFMA epilogue."""
    from ldnn.models.mlp import MLP
    torch.manual_seed(0)
    B = 1024
    m1, m2 = MLP(784, (1024, 512), 10, activation=act), MLP(784, (1024, 512), 10, activation=act)
    m2.load_state_dict(m1.state_dict())
    cfg = OptimConfig("sgd", lr=0.05, momentum=0.9)
    e1 = StaticMLPEngine(m1, B, cfg, use_graphs=True, library_gemms=True, library_dgrad=True)
    e2 = StaticMLPEngine(m2, B, cfg, use_graphs=True, library_gemms=True, library_dgrad=False)
    assert any(e1._lib_dgrad) and not any(e2._lib_dgrad)
    g = torch.Generator(device="cuda").manual_seed(5)
    l1, l2 = [], []
    for i in range(6):
        x = torch.randn(B, 784, device="cuda", generator=g).bfloat16()
        y = torch.randint(0, 10, (B,), device="cuda", generator=g)
        for e, ls in ((e1, l1), (e2, l2)):
            e.reset_stats()
            e.load_batch(x, y)
            e.step()
            ls.append(e.read_stats(B)[0])
    torch.cuda.synchronize()
    for a, b in zip(l1, l2):
        assert abs(a - b) < 1e-2 * max(1.0, abs(b)), (l1, l2)
    torch.testing.assert_close(e1.flat.master, e2.flat.master, rtol=2e-2, atol=2e-3)


def test_wgrad_q_splitk_matches_library_gemms():
    """Long-batch wgrads whose 256-tile grid is small (B = 4096, 1024-wide layers: 16
    tiles) run on gemm_q with split-K into slabs + slab_sum: after one step every weight
    gradient equals an fp32 reference on the engine's own backward tensors, and the
    ldnn-GEMM engine trains like the hipBLASLt-GEMM engine.  (The two engines' dz
    differ elementwise where bf16 ReLU masks flip, so they are not compared directly.)"""
    torch.manual_seed(0)
    B = 4096
    m1, m2 = mlp3(784, 1024, 10), mlp3(784, 1024, 10)
    m2.load_state_dict(m1.state_dict())
    cfg = OptimConfig("sgd", lr=0.05, momentum=0.0)
    e1 = StaticMLPEngine(m1, B, cfg, use_graphs=True, library_gemms=False)
    e2 = StaticMLPEngine(m2, B, cfg, use_graphs=True, library_gemms=True)
    assert e1._wgrad_slab[0] is not None and e1._wgrad_splitk[0] > 1   # split-K slabs + slab_sum
    g = torch.Generator(device="cuda").manual_seed(11)
    l1, l2 = [], []
    for i in range(6):
        x = torch.randn(B, 784, device="cuda", generator=g).bfloat16()
        y = torch.randint(0, 10, (B,), device="cuda", generator=g)
        for e, ls in ((e1, l1), (e2, l2)):
            e.reset_stats()
            e.load_batch(x, y)
            e.step()
            ls.append(e.read_stats(B)[0])
        if i == 0:
            torch.cuda.synchronize()
            for l in range(2):
                ref = e1.dz[l + 1].float().t() @ e1.h[l].float()
                err = (e1.dW[l] - ref).abs().max().item()
                assert err <= 1e-4 * ref.abs().max().item(), (l, err)
    for a, b in zip(l1, l2):
        assert abs(a - b) < 1e-2 * max(1.0, abs(b)), (l1, l2)


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_relu_masks_and_wgrad_slabs_match_plain_engine(opt):
    """The engine with ReLU bit masks (fwd writes, dgrad reads), the transposed-W dgrad
    and the first-layer bias gradient from the wgrad's ones column equals the engine
    reading the bf16 activations, k-strided W and dgrad-epilogue bias sums."""
    torch.manual_seed(0)
    B = 4096
    m1, m2 = mlp3(784, 1024, 10), mlp3(784, 1024, 10)
    m2.load_state_dict(m1.state_dict())
    cfg = OptimConfig(opt, lr=0.05 if opt == "sgd" else 1e-3, momentum=0.9)
    e1 = StaticMLPEngine(m1, B, cfg, use_graphs=True)
    e2 = StaticMLPEngine(m2, B, cfg, use_graphs=True, relu_masks=False, transposed_dgrad=False,
                         bias_ones_column=False)
    assert e1.mask[1] is not None and e1._wgrad_slab[0] is not None and e1.Wt[1] is not None
    assert e1._db0_from_wgrad and e1.xp.shape[1] == 792 and not e2._db0_from_wgrad
    assert e2.mask[1] is None and e2.Wt[1] is None
    g = torch.Generator(device="cuda").manual_seed(8)
    for _ in range(5):
        x = torch.randn(B, 784, device="cuda", generator=g).bfloat16()
        y = torch.randint(0, 10, (B,), device="cuda", generator=g)
        for e in (e1, e2):
            e.load_batch(x, y)
            e.step()
    torch.cuda.synchronize()
    # SGD: tight.  Adam: its m / sqrt(v) turns the bias gradients' different fp32 summation
    # order (MFMA ones column vs dgrad-epilogue sums) into up to ~lr-sized steps where a
    # gradient is near zero, so the bound is a fraction of the 5-step lr budget
    atol = 1e-5 if opt == "sgd" else 1e-3
    for p, q in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-4, atol=atol)




@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_eager_partial_batch_step_matches_reference(opt):
    """The trailing partial batch (StaticMLPEngine.eager_step: autograd on the engine's
    flat parameters + the fused update) == an fp32 torch step on that batch, and the
    next full engine step still matches (its accumulating gradients were left clean)."""
    torch.manual_seed(0)
    B, b = 512, 200
    m = mlp3(784, 256, 10)
    lin = [l for l in m.layers]
    ref = torch.nn.Sequential(torch.nn.Linear(784, 256), torch.nn.ReLU(), torch.nn.Linear(256, 256), torch.nn.ReLU(),
                              torch.nn.Linear(256, 10))
    with torch.no_grad():
        for r, l in zip([ref[0], ref[2], ref[4]], lin):
            r.weight.copy_(l.weight)
            r.bias.copy_(l.bias)
    ref = ref.cuda().float()
    cfg = OptimConfig(opt, lr=0.05 if opt == "sgd" else 1e-3, momentum=0.9)
    e = StaticMLPEngine(m, B, cfg, use_graphs=True)
    ropt = (torch.optim.SGD(ref.parameters(), lr=0.05, momentum=0.9) if opt == "sgd" else
            torch.optim.Adam(ref.parameters(), lr=1e-3))
    g = torch.Generator(device="cuda").manual_seed(4)
    for n in (B, b, B, B, b):
        x = torch.randn(n, 784, device="cuda", generator=g).bfloat16()
        y = torch.randint(0, 10, (n,), device="cuda", generator=g)
        if n == B:
            e.load_batch(x, y)
            e.step()
        else:
            e.eager_step(x, y)
        ropt.zero_grad()
        torch.nn.functional.cross_entropy(ref(x.float()), y).backward()
        ropt.step()
    torch.cuda.synchronize()
    for l, r in zip(lin, [ref[0], ref[2], ref[4]]):
        for p, q in ((l.weight, r.weight), (l.bias, r.bias)):
            torch.testing.assert_close(p.detach().float(), q.detach(), rtol=5e-2, atol=5e-3 if opt == "sgd" else 1e-2)  # Adam: sign-amplified bf16 noise near 0


@pytest.mark.parametrize("nproc,hops,weight", [(3, 1, None), (3, 1, 0.7), (3, 2, None), (3, 2, 0.6), (2, 2, None),
                                               (3, 0, 0.8), (4, 2, 0.5)])
def test_static_engine_per_step_gossip_and_weighted_match_reference_formulas(nproc, hops, weight):
    """--sync_every step --topology ring / double_ring (equal / weighted) and the weighted
    all-reduce on the static engine (grad_mix: per-bucket neighbour exchange between the
    backward's graph segments + the fused mix kernel) == the reference formulas
    (parallel.aggregation on FakeWorld, fp32) applied to the ranks' own gradients, step
    after step while the replicas drift apart (gloo ranks sharing the GPU)."""
    import os
    import socket
    import subprocess
    import sys

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", str(nproc), "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(root, "scripts", "check_engine_gossip.py"), "--hops", str(hops)]
    if weight is not None:
        cmd += ["--weight", str(weight)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "ENGINE_GOSSIP_OK" in r.stdout, r.stdout[-3000:]

