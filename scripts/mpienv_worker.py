import os, sys
sys.path.insert(0, sys.argv[1])
import torch
import ldnn
from ldnn.utils import distributed as D
ctx = D.setup("gloo", device="cpu", timeout_s=60)
t = torch.tensor([float(ctx.rank + 1)])
torch.distributed.all_reduce(t)
print(f"MPIENV rank={ctx.rank} world={ctx.world_size} local={ctx.local_rank} sum={t.item()}", flush=True)
D.teardown(ctx)
