"""The graph-captured static MLP engine trains like a plain PyTorch fp32 model."""
import pytest
import torch

import ldnn
from ldnn.models.mlp import mlp3
from ldnn.train.static_mlp import OptimConfig, StaticMLPEngine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("opt", ["sgd", "adam"])
@pytest.mark.parametrize("graphs", [False, True])
def test_engine_matches_fp32_reference(opt, graphs):
    torch.manual_seed(0)
    B = 256
    model = mlp3(784, 512, 10)
    ref = torch.nn.Sequential(torch.nn.Linear(784, 512), torch.nn.ReLU(), torch.nn.Linear(512, 512),
                              torch.nn.ReLU(), torch.nn.Linear(512, 10))
    for dst, src in zip(ref.parameters(), model.parameters()):
        dst.data.copy_(src.data)
    ref = ref.cuda()
    cfg = OptimConfig(opt, lr=0.05 if opt == "sgd" else 1e-3, momentum=0.9)
    eng = StaticMLPEngine(model, B, cfg, use_graphs=graphs)
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
